"""ctypes binding of libpekf.so (include/pekf.h).  No PyTorch, no CPU fallback.

The library is built in-tree (``poseestimationkf_amd/libpekf.so``, see csrc/Makefile or
``__graft_entry__.build()``).  If it is missing, importing this module raises: there is
no silent Python path for any operator.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

LIB_PATH = os.environ.get("PEKF_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "libpekf.so"))

PEKF_OK = 0
PEKF_ERR_INVALID = 1
PEKF_ERR_HIP = 2
PEKF_ERR_SINGULAR = 3
PEKF_ERR_NODEVICE = 4
PEKF_ERR_SVD = 5
PEKF_ERR_COMM = 6
PEKF_ERR_TIMEOUT = 7
MISSING_MAG_BIT = 0x80000000
RUN_MIXED_PRECISION = 0x1
RUN_STATE_SOA = 0x2
DT_ESCAPE = 0x7FFFFFFF
EV_TIME_EVENTS = 0x1
EV_F32_RECORDS = 0x2
EV_F64_EVENTS = 0x4
WIRE_FRAME_ROWS = 0x1


class PekfError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__("libpekf status %d: %s" % (status, msg))
        self.status = status


class NoDeviceError(PekfError):
    pass


class CommTimeoutError(PekfError):
    """A collective step passed its deadline (PEKF_COMM_TIMEOUT_S); the communicator was aborted.

    After a communicator-creation timeout the process must exit (os._exit: the abandoned RCCL init
    thread still holds RCCL's bootstrap state); until it does, every later creation fails at once."""


_i64, _u32, _int, _dbl, _sz, _vp = ctypes.c_int64, ctypes.c_uint32, ctypes.c_int, ctypes.c_double, ctypes.c_size_t, ctypes.c_void_p
_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int)

# name -> argtypes (every function returns int status unless listed in _RESTYPE)
SIGNATURES = {
    "pekf_abi_version": [],
    "pekf_last_error": [],
    "pekf_device_count": [_ip],
    "pekf_set_device": [_int],
    "pekf_get_device": [_ip],
    "pekf_device_name": [_int, ctypes.c_char_p, _int],
    "pekf_malloc": [ctypes.POINTER(_vp), _sz],
    "pekf_free": [_vp],
    "pekf_memcpy_h2d": [_vp, _vp, _sz, _vp],
    "pekf_memcpy_d2h": [_vp, _vp, _sz, _vp],
    "pekf_memcpy_d2d": [_vp, _vp, _sz, _vp],
    "pekf_memset": [_vp, _int, _sz, _vp],
    "pekf_stream_create": [ctypes.POINTER(_vp)],
    "pekf_stream_destroy": [_vp],
    "pekf_stream_sync": [_vp],
    "pekf_device_sync": [],
    "pekf_set_percall_mode": [_int],
    "pekf_get_percall_mode": [ctypes.POINTER(_int)],
    "pekf_event_create": [ctypes.POINTER(_vp)],
    "pekf_event_destroy": [_vp],
    "pekf_event_record": [_vp, _vp],
    "pekf_event_sync": [_vp],
    "pekf_event_elapsed_ms": [ctypes.POINTER(ctypes.c_float), _vp, _vp],
    "pekf_rk4": [_i64, _vp, _vp, _vp, _vp],
    "pekf_rk4_dev": [_i64, _vp, _vp, _vp, _vp, _vp],
    "pekf_norm": [_i64, _i64, _vp, _vp],
    "pekf_jacobian_a": [_i64, _vp, _vp],
    "pekf_jacobian_b": [_i64, _vp, _vp],
    "pekf_comparator": [_i64, _vp, _vp, _vp],
    "pekf_predict": [_i64] + [_vp] * 9,
    "pekf_predict_dev": [_i64] + [_vp] * 9 + [_vp, _vp],
    "pekf_correct": [_i64] + [_vp] * 9,
    "pekf_correct_dev": [_i64] + [_vp] * 9 + [_vp],
    "pekf_wahba_rotation": [_i64] + [_vp] * 7,
    "pekf_wahba_quaternion": [_i64] + [_vp] * 7,
    "pekf_rotmat_to_quat": [_i64, _vp, _vp],
    "pekf_run_dev": [_i64, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _dbl, _dbl, _vp, _vp, _u32, _vp],
    "pekf_run_rec64_dev": [_i64, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _dbl, _dbl, _vp, _vp, _vp],
    "pekf_run_ext_dev": [_i64, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _dbl, _dbl, _vp, _vp, _u32,
                         _vp],
    "pekf_reset_state_dev": [_i64, _vp, _vp, _vp],
    "pekf_state_layout_dev": [_i64, _vp, _vp, _vp, _vp, _int, _vp],
    "pekf_filter_create": [_i64, _vp, _vp, _dbl, _dbl, _vp, _u32, ctypes.POINTER(_vp)],
    "pekf_filter_destroy": [_vp],
    "pekf_filter_set_state": [_vp, _vp, _vp],
    "pekf_filter_get_state": [_vp, _vp, _vp],
    "pekf_filter_set_time": [_vp, _vp],
    "pekf_filter_get_time": [_vp, _vp],
    "pekf_filter_device_state": [_vp, ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_vp)],
    "pekf_filter_update": [_vp] * 7,
    "pekf_filter_update_dev": [_vp] * 8,
    "pekf_filter_run": [_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp],
    "pekf_filter_run_ext": [_vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "pekf_gyro_chain_dev": [_i64, _i64, _i64, _i64, _vp, _vp, _vp, _vp],
    "pekf_gyro_chain_ext_dev": [_i64, _i64, _i64, _i64, _vp, _vp, _vp, _vp, _vp],
    "pekf_wahba_stream_dev": [_i64, _i64, _i64, _i64, _vp, _vp, _vp, _dbl, _dbl, _vp, _vp],
    "pekf_quat_to_rpy": [_i64, _vp, _vp],
    "pekf_gyro_chain_rec64_dev": [_i64, _i64, _i64, _i64, _vp, _vp, _vp, _vp],
    "pekf_wahba_stream_rec64_dev": [_i64, _i64, _i64, _i64, _vp, _vp, _vp, _dbl, _dbl, _vp, _vp],
    "pekf_frontend_dev": [_i64, _i64, _vp, _vp, _vp, _dbl, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "pekf_frontend_ext_dev": [_i64, _i64, _vp, _vp, _vp, _dbl, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _u32, _vp, _vp],
    "pekf_frontend_init_dev": [_i64, _i64, _vp, _vp, _int, _vp, _vp, _vp, _vp, _vp],
    "pekf_frontend_init_ext_dev": [_i64, _i64, _vp, _vp, _int, _vp, _vp, _vp, _vp, _u32, _vp],
    "pekf_f32_wire_values": [_i64, _vp, _vp],
    "pekf_wire_parse": [ctypes.c_char_p, _i64, _i64, _vp, _vp, _vp, _vp, ctypes.POINTER(_i64)],
    "pekf_wire_events_dev": [_i64, _i64, _vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "pekf_wire_events_ext_dev": [_i64, _i64, _vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _u32, _vp],
    "pekf_live_dev": [_i64, _i64, _vp, _vp, _vp, _dbl, _vp, _vp, _dbl, _dbl, _vp, _vp, _vp, _vp],
    "pekf_live_ext_dev": [_i64, _i64, _vp, _vp, _vp, _dbl, _vp, _vp, _dbl, _dbl, _vp, _vp, _u32, _vp, _vp],
    "pekf_log_scan": [ctypes.c_char_p, ctypes.POINTER(_i64)],
    "pekf_log_read": [ctypes.c_char_p, _i64, _vp, _vp, _vp, _vp, _dp, _dp, _dp],
    "pekf_log_read_ext": [ctypes.c_char_p, _i64, _vp, _vp, _vp, _vp, _vp, ctypes.POINTER(_i64), _dp, _dp, _dp],
    "pekf_log_read64": [ctypes.c_char_p, _i64, _vp, _vp, _vp, _vp, _dp, _dp, _dp],
    "pekf_log_write": [ctypes.c_char_p, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "pekf_quat_to_rpy_dev": [_i64, _vp, _vp, _vp],
    "pekf_synth_dev": [_i64, _i64, _i64, _u32, _int, _dp, _dbl, _vp, _vp, _vp, _vp, _vp],
    "pekf_comm_version": [_ip],
    "pekf_comm_unique_id": [ctypes.c_char_p],
    "pekf_comm_init": [ctypes.c_char_p, _int, _int, ctypes.POINTER(_vp)],
    "pekf_comm_init_timeout": [ctypes.c_char_p, _int, _int, _dbl, ctypes.POINTER(_vp)],
    "pekf_comm_abort": [_vp],
    "pekf_comm_wait": [_vp, _vp, _dbl],
    "pekf_comm_init_all": [_int, _ip, ctypes.POINTER(_vp)],
    "pekf_comm_init_all_timeout": [_int, _ip, _dbl, ctypes.POINTER(_vp)],
    "pekf_comm_destroy": [_vp],
    "pekf_comm_rank": [_vp, _ip, _ip, _ip],
    "pekf_gather_dev": [_vp, _vp, _i64, _vp, _int, _vp],
    "pekf_gather_multi_dev": [_int, ctypes.POINTER(_vp), ctypes.POINTER(_vp), _i64, _vp, _int, ctypes.POINTER(_vp)],
    "pekf_allreduce_max_dev": [_vp, _vp, _i64, _vp],
}
_RESTYPE = {"pekf_abi_version": ctypes.c_int, "pekf_last_error": ctypes.c_char_p}


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            "libpekf.so not found at %s -- build it first (python -c 'import __graft_entry__ as g; g.build()' "
            "or make -C poseestimationkf_amd/csrc). There is no CPU fallback." % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    for name, argtypes in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = _RESTYPE.get(name, ctypes.c_int)
    if lib.pekf_abi_version() != 1:
        raise ImportError("libpekf ABI mismatch")
    return lib


lib = _load()


def last_error():
    return (lib.pekf_last_error() or b"").decode(errors="replace")


def check(status):
    if status == PEKF_OK:
        return
    msg = last_error()
    if status == PEKF_ERR_SINGULAR:
        raise np.linalg.LinAlgError(msg or "Singular matrix")
    if status == PEKF_ERR_SVD:
        raise np.linalg.LinAlgError(msg or "SVD did not converge")
    if status == PEKF_ERR_NODEVICE:
        raise NoDeviceError(status, msg)
    if status == PEKF_ERR_TIMEOUT:
        raise CommTimeoutError(status, msg)
    raise PekfError(status, msg)


def device_count():
    n = ctypes.c_int(0)
    check(lib.pekf_device_count(ctypes.byref(n)))
    return n.value


def dptr(a):
    """float64 C-contiguous host array -> double*"""
    return a.ctypes.data_as(_dp)


def f64(a, shape):
    """Convert list / ndarray input to a fresh C-contiguous float64 array of the given shape."""
    out = np.array(a, dtype=np.float64, copy=True, order="C")
    return out.reshape(shape)
