"""ctypes binding of `include/mano_hip.h` (the C-ABI of libmano_hip.so).

Loads the in-tree gfx950 library; there is no fallback: if the library is
missing or fails to load, `lib()` raises `MissingExtensionError` so a product
call can never silently run anything else.
"""
from __future__ import annotations

import ctypes
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libmano_hip.so")
HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(HERE)), "include", "mano_hip.h")

MANO_OK, MANO_EINVAL, MANO_EHIP, MANO_ESMALL, MANO_ESTATE, MANO_ECOMM, MANO_EDEVICE = 0, -1, -2, -3, -4, -5, -6
MANO_MEMCPY_HOST_TO_DEVICE, MANO_MEMCPY_DEVICE_TO_HOST, MANO_MEMCPY_DEVICE_TO_DEVICE = 1, 2, 3
MANO_COMM_ID_BYTES = 128
MANO_PRECISION_FP32, MANO_PRECISION_F16X3 = 0, 1
MANO_DEVICE_SKIN_HANDOFF_TIMEOUT = 1
MANO_STATUS_CLEAR, MANO_STATUS_NO_WAIT = 1, 2
ABI_VERSION = 7
PRECISIONS = {"fp32": MANO_PRECISION_FP32, "f16x3": MANO_PRECISION_F16X3}
_CODE_NAMES = {MANO_EINVAL: "MANO_EINVAL", MANO_EHIP: "MANO_EHIP", MANO_ESMALL: "MANO_ESMALL",
               MANO_ESTATE: "MANO_ESTATE", MANO_ECOMM: "MANO_ECOMM", MANO_EDEVICE: "MANO_EDEVICE"}


class MissingExtensionError(RuntimeError):
    """libmano_hip.so is not built / not loadable: the HIP path cannot run."""


class ManoError(RuntimeError):
    def __init__(self, code, message):
        super().__init__(f"{_CODE_NAMES.get(code, code)}: {message}")
        self.code = code


class DeviceStatusError(ManoError):
    """A kernel raised a MANO_DEVICE_* bit: some launch's outputs are not
    valid.  Raised by a wrapper that read the status (`status` = the bits), and
    by any launching call while the bit is still set (MANO_EDEVICE)."""

    def __init__(self, status, message=None):
        names = [n for n, b in (("MANO_DEVICE_SKIN_HANDOFF_TIMEOUT", MANO_DEVICE_SKIN_HANDOFF_TIMEOUT),)
                 if status & b]
        super().__init__(MANO_EDEVICE, message or
                         f"device status 0x{status:x} ({', '.join(names) or 'unknown bits'})")
        self.status = status


_p = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32
_dptr = ctypes.POINTER(ctypes.c_double)
_ipt = ctypes.POINTER(ctypes.c_int32)

# name -> (restype, argtypes); mirrors include/mano_hip.h one to one.
SIGNATURES = {
    "mano_abi_version": (ctypes.c_int, []),
    "mano_last_error": (ctypes.c_char_p, []),
    "mano_model_create": (ctypes.c_int, [ctypes.c_int, _i32, _dptr, _dptr, _dptr, _dptr, _dptr,
                                         _ipt, _dptr, _dptr, ctypes.POINTER(_p)]),
    "mano_model_destroy": (ctypes.c_int, [_p]),
    "mano_model_set_precision": (ctypes.c_int, [_p, _i32]),
    "mano_model_get_precision": (ctypes.c_int, [_p, ctypes.POINTER(_i32)]),
    "mano_model_info": (ctypes.c_int, [_p, ctypes.POINTER(_i32), ctypes.POINTER(_i32)]),
    "mano_model_device_status": (ctypes.c_int, [_p, ctypes.POINTER(_i32), _i32]),
    "mano_workspace_bytes": (ctypes.c_size_t, [_p, _i64]),
    "mano_forward_workspace_bytes": (ctypes.c_size_t, [_p, _i64]),
    "mano_workspace_offsets": (ctypes.c_int, [_p, _i64, ctypes.POINTER(ctypes.c_size_t),
                                              ctypes.POINTER(ctypes.c_size_t),
                                              ctypes.POINTER(ctypes.c_size_t)]),
    "mano_forward": (ctypes.c_int, [_p, _i64, _p, _i64, _p, _p, _p, _p, _p, _p, _p, _p,
                                    ctypes.c_size_t, _p]),
    "mano_stage_articulate": (ctypes.c_int, [_p, _i64, _p, _i64, _p, _p, _p, _p, _p, _p,
                                             ctypes.c_size_t, _p]),
    "mano_stage_blend": (ctypes.c_int, [_p, _i64, _p, _p, ctypes.c_size_t, _p]),
    "mano_stage_skin": (ctypes.c_int, [_p, _i64, _p, _p, _p, _p, ctypes.c_size_t, _p]),
    "mano_stage_blend_skin": (ctypes.c_int, [_p, _i64, _p, _p, _p, _p, ctypes.c_size_t, _p]),
    "mano_pose_from_pca": (ctypes.c_int, [_p, _i64, _p, _i32, _i64, _p, _i64, _p, _p]),
    "mano_forward_pca": (ctypes.c_int, [_p, _i64, _p, _i64, _p, _i32, _i64, _p, _i64, _p, _p, _p,
                                        _p, _p, _p, _p, _p, ctypes.c_size_t, _p]),
    "mano_rodrigues": (ctypes.c_int, [ctypes.c_int, _i64, _p, _p, _p]),
    "mano_alloc": (ctypes.c_int, [ctypes.c_int, ctypes.c_size_t, ctypes.POINTER(_p)]),
    "mano_free": (ctypes.c_int, [ctypes.c_int, _p]),
    "mano_host_alloc": (ctypes.c_int, [ctypes.c_size_t, ctypes.POINTER(_p)]),
    "mano_host_free": (ctypes.c_int, [_p]),
    "mano_memcpy": (ctypes.c_int, [ctypes.c_int, _p, _p, ctypes.c_size_t, _i32, _p]),
    "mano_synchronize": (ctypes.c_int, [ctypes.c_int]),
    "mano_synthetic_inputs": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint64, _i64, _i64, ctypes.c_float,
                                             ctypes.c_float, ctypes.c_float, _p, _p, _p, _p]),
    "mano_comm_unique_id": (ctypes.c_int, [ctypes.c_char_p]),
    "mano_comm_create": (ctypes.c_int, [ctypes.c_int, _i32, _i32, ctypes.c_char_p, ctypes.POINTER(_p)]),
    "mano_comm_create_all": (ctypes.c_int, [_i32, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(_p)]),
    "mano_group_start": (ctypes.c_int, []),
    "mano_group_end": (ctypes.c_int, []),
    "mano_comm_destroy": (ctypes.c_int, [_p]),
    "mano_gather": (ctypes.c_int, [_p, _p, ctypes.c_size_t, _p, ctypes.POINTER(ctypes.c_size_t), _i32, _p]),
    "mano_allgather": (ctypes.c_int, [_p, _p, ctypes.c_size_t, _p, _p]),
    "mano_gather_check": (ctypes.c_int, [_p, _p, ctypes.c_size_t, _p, ctypes.POINTER(ctypes.c_size_t), _i32]),
    "mano_comm_info": (ctypes.c_int, [_p, ctypes.POINTER(_i32), ctypes.POINTER(_i32), ctypes.POINTER(_i32)]),
}

_LIB = None


def header_functions(path: str = HEADER_PATH):
    """Names of every function the public header declares."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mano_[a-z_]+)\s*\(", text)))


def lib() -> ctypes.CDLL:
    """Load libmano_hip.so once (RTLD_GLOBAL off) and declare every signature."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise MissingExtensionError(
            f"{LIB_PATH} is not built; run `make -C mano-hand_amd` or "
            "`python -c 'import __graft_entry__ as g; g.build()'`")
    try:
        # torch (if imported) already holds libamdhip64.so.7; the same SONAME
        # resolves to that copy, so torch and this library share one HIP runtime.
        handle = ctypes.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover - depends on the box
        raise MissingExtensionError(f"cannot load {LIB_PATH}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(handle, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = handle
    return _LIB


def check(rc: int) -> None:
    if rc != MANO_OK:
        msg = lib().mano_last_error()
        msg = msg.decode() if msg else ""
        if rc == MANO_EDEVICE:
            m = re.search(r"device status 0x([0-9a-f]+)", msg)
            raise DeviceStatusError(int(m.group(1), 16) if m else 0, msg)
        raise ManoError(rc, msg)


def last_error() -> str:
    msg = lib().mano_last_error()
    return msg.decode() if msg else ""


class _PointerAttributes(ctypes.Structure):
    """hipPointerAttribute_t (hip_runtime_api.h)."""
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int), ("devicePointer", ctypes.c_void_p),
                ("hostPointer", ctypes.c_void_p), ("isManaged", ctypes.c_int), ("allocationFlags", ctypes.c_uint)]


_HIP_MEMORY_TYPE_HOST = 1


def host_block_mapped(ptr: int) -> bool:
    """True when `ptr` is pinned host memory that the HIP runtime maps into
    the device address space at the same address (hipHostMalloc'd, e.g.
    torch's pinned tensors), so kernels may read and write it directly."""
    # the HIP runtime libmano_hip.so is linked against (dlsym on the
    # library's handle searches its dependencies): never a second copy
    try:
        get_attrs = lib().hipPointerGetAttributes
        get_last = lib().hipGetLastError
    except AttributeError:
        return False
    a = _PointerAttributes()
    rc = get_attrs(ctypes.byref(a), ctypes.c_void_p(ptr))
    if rc != 0:
        get_last()  # this query's error is not the caller's
        return False
    return a.type == _HIP_MEMORY_TYPE_HOST and a.devicePointer == ptr
