"""poseestimationkf_amd -- MI355X-native batched quaternion EKF (predict + Wahba + update).

Layout
  csrc/        HIP kernels for gfx950 + the C ABI of include/pekf.h  -> libpekf.so
  _lib.py      ctypes binding (no PyTorch; raises if libpekf.so is missing)
  engine.py    device buffers, resident IMU windows, BatchedEKF (fused kernel), batched per-call ops
  dropin/      ExtendedKalmanFilter / Wahba / UtilityFunctions / ReadFile with the reference's API
  synth.py     host mirror of the device Philox IMU generator (bit-identical)
  logformat.py the live server's text log (emit / ingest)
  shard.py     filter-batch sharding over ranks + the final-quaternion gather

``engine`` (and anything that touches the GPU) is imported on demand so the host-only
modules work on machines without the built library.
"""
__version__ = "0.1.0"


def __getattr__(name):
    if name in ("engine", "_lib", "shard"):
        import importlib
        return importlib.import_module("." + name, __name__)
    raise AttributeError(name)
