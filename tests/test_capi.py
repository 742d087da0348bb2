"""CPU-side checks of the C ABI: the library loads, exports every declared symbol, and the
product path refuses to compute without a device (no CPU fallback)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from .conftest import ROOT

HEADER = os.path.join(ROOT, "include", "pekf.h")


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(pekf_\w+)\s*\(", text, re.M)))


def test_header_declares_the_replaced_reference_interfaces():
    syms = declared_symbols()
    for s in ("pekf_predict", "pekf_correct", "pekf_rk4", "pekf_jacobian_a", "pekf_jacobian_b",
              "pekf_comparator", "pekf_norm", "pekf_wahba_rotation", "pekf_wahba_quaternion",
              "pekf_rotmat_to_quat", "pekf_run_dev", "pekf_synth_dev"):
        assert s in syms
    assert len(syms) >= 35


def test_library_exports_every_declared_symbol():
    from poseestimationkf_amd import _lib
    syms = declared_symbols()
    missing = [s for s in syms if not hasattr(_lib.lib, s)]
    assert not missing, missing
    assert set(syms) == set(_lib.SIGNATURES), set(syms) ^ set(_lib.SIGNATURES)
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (pekf_\w+)", out))
    assert set(syms) <= exported
    assert _lib.lib.pekf_abi_version() == 1


def test_library_is_gfx950_code_object():
    from poseestimationkf_amd import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_no_cpu_fallback_without_device():
    from poseestimationkf_amd import _lib
    if _lib.device_count() > 0:
        pytest.skip("a device is visible")
    from poseestimationkf_amd import engine
    with pytest.raises(_lib.NoDeviceError):
        engine.rk4(np.array([1.0, 0, 0, 0]), 1e7, np.zeros(3))
    with pytest.raises(_lib.NoDeviceError):
        engine.BatchedEKF(4)
    with pytest.raises(_lib.NoDeviceError):
        engine.FilterHandle(np.zeros((4, 3)), np.zeros((4, 3)))
    from poseestimationkf_amd import _fastcall
    with pytest.raises(_lib.NoDeviceError):
        _fastcall.predict([0.1, 0.2, 0.3], 1e7, np.array([1.0, 0, 0, 0]), np.eye(4), np.eye(3), np.eye(4))
    p = ctypes.c_void_p()
    assert _lib.lib.pekf_malloc(ctypes.byref(p), 64) == _lib.PEKF_ERR_NODEVICE
    assert "no HIP device" in _lib.last_error()
    from poseestimationkf_amd import shard  # the collective refuses too (RCCL is never loaded)
    with pytest.raises(_lib.NoDeviceError):
        shard.Communicator.unique_id()
    with pytest.raises(_lib.NoDeviceError):
        shard.Communicator(bytes(128), 1, 0)


def test_fastcall_binding_checks_shapes():
    from poseestimationkf_amd import _fastcall
    with pytest.raises(ValueError, match="gyro"):
        _fastcall.predict([0.1, 0.2], 1e7, np.zeros(4), np.eye(4), np.eye(3), np.eye(4))
    with pytest.raises(ValueError, match="mag0"):
        _fastcall.correct(np.zeros(3), np.zeros(3), np.zeros(4), np.eye(4), np.eye(4), np.zeros(3), np.zeros(2))
    with pytest.raises(TypeError):
        _fastcall.wahba_quaternion(np.zeros(3))


def test_invalid_arguments_are_reported_not_crashed():
    from poseestimationkf_amd import _lib
    h = ctypes.c_void_p()
    assert _lib.lib.pekf_comm_init(bytes(128), 2, 2, ctypes.byref(h)) == _lib.PEKF_ERR_INVALID  # rank >= nranks
    assert "rank" in _lib.last_error()
    assert _lib.lib.pekf_gather_dev(None, None, 4, None, 0, None) == _lib.PEKF_ERR_INVALID
    assert _lib.lib.pekf_comm_destroy(None) == _lib.PEKF_OK
    st = _lib.lib.pekf_run_dev(-1, 1, 1, 0, None, None, None, None, None, None, 1.0, 0.1, None, None, 0, None)
    assert st == _lib.PEKF_ERR_INVALID and "negative" in _lib.last_error()
    st = _lib.lib.pekf_run_dev(4, 1, 1, 0, None, None, None, None, None, None, 1.0, 0.1, None, None, 0, None)
    assert st == _lib.PEKF_ERR_INVALID and "null" in _lib.last_error()
    st = _lib.lib.pekf_run_dev(4, 1, 1, 0, None, None, None, None, None, None, 1.0, 0.1, None, None, 0x4, None)
    assert st == _lib.PEKF_ERR_INVALID and "flags" in _lib.last_error()
    st = _lib.lib.pekf_live_dev(-1, 8, None, None, None, 0.1, None, None, 1.0, 0.1, None, None, None, None)
    assert st == _lib.PEKF_ERR_INVALID and "negative" in _lib.last_error()
    st = _lib.lib.pekf_live_dev(4, 8, None, None, None, 0.1, None, None, 1.0, 0.1, None, None, None, None)
    assert st == _lib.PEKF_ERR_INVALID and "null" in _lib.last_error()
    st = _lib.lib.pekf_state_layout_dev(4, None, None, None, None, 1, None)
    assert st == _lib.PEKF_ERR_INVALID and "null" in _lib.last_error()
    h = ctypes.c_void_p()
    st = _lib.lib.pekf_filter_create(0, None, None, 1.0, 0.1, None, 0, ctypes.byref(h))
    assert st == _lib.PEKF_ERR_INVALID and "batch" in _lib.last_error() and not h.value
    st = _lib.lib.pekf_filter_create(4, None, None, 1.0, 0.1, None, 0, ctypes.byref(h))
    assert st == _lib.PEKF_ERR_INVALID and "null" in _lib.last_error()
    assert _lib.lib.pekf_filter_destroy(None) == _lib.PEKF_OK
    st = _lib.lib.pekf_filter_update(None, None, None, None, None, None, None)
    assert st == _lib.PEKF_ERR_INVALID and "handle" in _lib.last_error()


def test_product_package_never_imports_the_oracle():
    pkg = os.path.join(ROOT, "poseestimationkf_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".hpp", ".cpp")):
                src = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle|ekf_oracle|oracle_c|ekf_numpy", src, re.M), f


def test_round3_entry_points_check_their_arguments():
    """The dt-escape / time-event entry points validate before touching a device (CPU)."""
    from poseestimationkf_amd import _lib
    L = _lib.lib
    st = L.pekf_run_ext_dev(4, 2, 1, 0, None, None, None, None, None, None, None, 1.0, 0.1, None, None, 0, None)
    assert st == _lib.PEKF_ERR_INVALID and "null" in _lib.last_error()
    st = L.pekf_run_ext_dev(4, 2, 1, 0, 16, 16, 8, 4, 8, 8, 8, 1.0, 0.1, None, None, 0, None)  # dt_ext % 8 != 0
    assert st == _lib.PEKF_ERR_INVALID and "misaligned" in _lib.last_error()
    assert L.pekf_run_ext_dev(0, 5, 1, 0, None, None, None, None, None, None, None, 1.0, 0.1, None, None, 0,
                              None) == _lib.PEKF_OK                                     # empty batch: no-op
    st = L.pekf_frontend_ext_dev(4, 8, None, None, None, 0.1, 3, None, None, None, None, None, None, 0x2, None, None)
    assert st == _lib.PEKF_ERR_INVALID and "flags" in _lib.last_error()
    st = L.pekf_frontend_ext_dev(4, 8, None, None, None, 0.1, 3, None, None, None, None, None, None, 0x1, None, None)
    assert st == _lib.PEKF_ERR_INVALID and "null" in _lib.last_error()
    st = L.pekf_live_ext_dev(4, 8, None, None, None, 0.1, None, None, 1.0, 0.1, None, None, 0x8, None, None)
    assert st == _lib.PEKF_ERR_INVALID and "flags" in _lib.last_error()
    st = L.pekf_live_ext_dev(-1, 8, None, None, None, 0.1, None, None, 1.0, 0.1, None, None, 0, None, None)
    assert st == _lib.PEKF_ERR_INVALID and "negative" in _lib.last_error()
    st = L.pekf_log_read_ext(b"/nonexistent", 1, None, None, None, None, None, None, None, None, None)
    assert st == _lib.PEKF_ERR_INVALID and "null" in _lib.last_error()
    h = ctypes.c_void_p()
    st = L.pekf_filter_run_ext(None, 2, 1, 0, None, None, None, None, None, None, None)
    assert st == _lib.PEKF_ERR_INVALID and "handle" in _lib.last_error()
    assert h.value is None


def test_round4_entry_points_check_their_arguments():
    """The collective deadlines and the escaped-dt gyro chain validate before touching a device (CPU)."""
    from poseestimationkf_amd import _lib
    L = _lib.lib
    h = ctypes.c_void_p()
    assert L.pekf_comm_init_timeout(bytes(128), 2, 5, 10.0, ctypes.byref(h)) == _lib.PEKF_ERR_INVALID
    assert "rank" in _lib.last_error() and not h.value
    assert L.pekf_comm_wait(None, None, 1.0) == _lib.PEKF_ERR_INVALID and "communicator" in _lib.last_error()
    assert L.pekf_comm_abort(None) == _lib.PEKF_OK
    st = L.pekf_gyro_chain_ext_dev(4, 8, 4, 0, None, None, None, None, None)
    assert st == _lib.PEKF_ERR_INVALID and "null" in _lib.last_error()
    st = L.pekf_gyro_chain_ext_dev(4, 1 << 31, 4, 0, 16, None, 16, None, None)
    assert st == _lib.PEKF_ERR_INVALID and "2^31" in _lib.last_error()
    assert L.pekf_gyro_chain_ext_dev(0, 8, 4, 0, None, None, None, None, None) == _lib.PEKF_OK   # empty batch
    st = L.pekf_live_ext_dev(4, 1 << 30, 16, 16, 16, 0.1, 16, 16, 1.0, 0.1, 16, 16, 0, None, None)
    assert st == _lib.PEKF_ERR_INVALID and "2^30" in _lib.last_error()
    st = L.pekf_frontend_init_dev(4, 1 << 30, 16, 16, 100, 16, 16, None, 16, None)
    assert st == _lib.PEKF_ERR_INVALID and "2^30" in _lib.last_error()
    assert _lib.PEKF_ERR_TIMEOUT == 7 and issubclass(_lib.CommTimeoutError, _lib.PekfError)
    with pytest.raises(_lib.CommTimeoutError):
        _lib.check(_lib.PEKF_ERR_TIMEOUT)
