"""The torch-free binding's status handling (integration/mano_hip_ffi.py), on
CPU with the library's status call replaced: a raised MANO_DEVICE_* bit is
reported once and TAKEN (MANO_STATUS_CLEAR), so the Engine stays usable --
left set, every later launch on the model would return MANO_EDEVICE."""
import ctypes
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "integration"))


def test_status_reported_once_then_cleared():
    import mano_hip_ffi as ffi
    flags_seen, state = [], {"bits": 1}

    def fake_status(h, st_ptr, flags):
        flags_seen.append(flags)
        ctypes.cast(st_ptr, ctypes.POINTER(ctypes.c_int32))[0] = state["bits"]
        if flags & ffi.STATUS_CLEAR:
            state["bits"] = 0
        return 0

    class FakeLib:
        mano_model_device_status = staticmethod(fake_status)

    eng = ffi.Engine.__new__(ffi.Engine)
    eng._h = ctypes.c_void_p(1)
    real = ffi._lib
    ffi._lib = FakeLib()
    try:
        with pytest.raises(RuntimeError, match="device status 0x1"):
            eng._check_status()
        assert any(f & ffi.STATUS_CLEAR for f in flags_seen)        # taken when reported
        assert all(f & ffi.STATUS_NO_WAIT for f in flags_seen)      # the caller already synced
        eng._check_status()                                          # nothing left: no raise
    finally:
        ffi._lib = real
