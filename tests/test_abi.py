"""The C-ABI library loads, exports every symbol include/mano_hip.h declares,
and rejects bad arguments with status codes -- all without touching a GPU."""
import ctypes
import os

import pytest

from conftest import REPO
from mano_amd import _abi


def test_library_exports_every_header_symbol():
    lib = _abi.lib()
    names = _abi.header_functions()
    assert len(names) >= 13
    for n in names:
        assert hasattr(lib, n), n
        assert n in _abi.SIGNATURES, f"{n} declared in the header but not bound"
    assert set(_abi.SIGNATURES) == set(names)
    assert lib.mano_abi_version() == _abi.ABI_VERSION == 7


@pytest.mark.parametrize("cc,lang", [("g++", "c++"), ("gcc", "c")])
def test_header_compiles_alone(cc, lang):
    """include/mano_hip.h is self-contained C and C++ (a stray comment
    terminator once left prose outside the comment and broke every build)."""
    import shutil
    import subprocess
    if shutil.which(cc) is None:
        pytest.skip(f"{cc} not installed")
    r = subprocess.run([cc, "-fsyntax-only", "-Wall", "-Werror", "-x", lang, _abi.HEADER_PATH],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_library_is_gfx950_code_object():
    data = open(_abi.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_create_rejects_bad_arguments():
    lib = _abi.lib()
    out = ctypes.c_void_p()
    assert lib.mano_model_create(-1, 778, None, None, None, None, None, None, None, None,
                                 ctypes.byref(out)) == _abi.MANO_EINVAL
    assert "negative" in _abi.last_error()
    assert lib.mano_model_create(0, 778, None, None, None, None, None, None, None, None,
                                 None) == _abi.MANO_EINVAL
    assert lib.mano_model_create(0, 0, None, None, None, None, None, None, None, None,
                                 ctypes.byref(out)) == _abi.MANO_EINVAL
    assert out.value is None


def test_null_handle_paths():
    lib = _abi.lib()
    assert lib.mano_workspace_bytes(None, 10) == 0
    assert lib.mano_model_destroy(None) == _abi.MANO_OK
    assert lib.mano_forward(None, 1, None, 10, None, None, None, None, None, None, None, None,
                            0, None) == _abi.MANO_EINVAL
    assert "NULL" in _abi.last_error()
    for fn, args in (("mano_stage_blend", (None, 1, None, None, 0, None)),
                     ("mano_stage_skin", (None, 1, None, None, None, None, 0, None)),
                     ("mano_pose_from_pca", (None, 1, None, 9, 9, None, 0, None, None))):
        assert getattr(lib, fn)(*args) == _abi.MANO_EINVAL


def test_rodrigues_argument_checks():
    lib = _abi.lib()
    assert lib.mano_rodrigues(0, 0, None, None, None) == _abi.MANO_OK  # empty: no launch
    assert lib.mano_rodrigues(0, -1, None, None, None) == _abi.MANO_EINVAL
    assert lib.mano_rodrigues(-1, 4, ctypes.c_void_p(16), ctypes.c_void_p(16), None) == _abi.MANO_EINVAL


def test_check_raises_with_message():
    lib = _abi.lib()
    rc = lib.mano_forward(None, 1, None, 10, None, None, None, None, None, None, None, None, 0, None)
    with pytest.raises(_abi.ManoError) as ei:
        _abi.check(rc)
    assert ei.value.code == _abi.MANO_EINVAL


def test_memory_and_workload_argument_checks():
    """The framework-free memory calls refuse bad arguments before any HIP call."""
    lib = _abi.lib()
    assert lib.mano_alloc(0, 16, None) == _abi.MANO_EINVAL
    out = ctypes.c_void_p()
    assert lib.mano_alloc(-1, 16, ctypes.byref(out)) == _abi.MANO_EINVAL and out.value is None
    assert lib.mano_free(0, None) == _abi.MANO_OK
    assert lib.mano_memcpy(0, ctypes.c_void_p(16), ctypes.c_void_p(16), 4, 9, None) == _abi.MANO_EINVAL
    assert "kind" in _abi.last_error()
    assert lib.mano_memcpy(0, None, ctypes.c_void_p(16), 4, _abi.MANO_MEMCPY_HOST_TO_DEVICE,
                           None) == _abi.MANO_EINVAL
    assert lib.mano_memcpy(0, None, None, 0, _abi.MANO_MEMCPY_HOST_TO_DEVICE, None) == _abi.MANO_OK
    assert lib.mano_synchronize(-1) == _abi.MANO_EINVAL
    assert lib.mano_synthetic_inputs(0, 1, -1, 4, 1.0, 0.5, 1.0, None, None, None, None) == _abi.MANO_EINVAL
    assert lib.mano_synthetic_inputs(0, 1, 0, 0, 1.0, 0.5, 1.0, None, None, None, None) == _abi.MANO_OK


def test_forward_pca_and_comm_argument_checks():
    lib = _abi.lib()
    assert lib.mano_forward_pca(None, 1, None, 10, None, 9, 9, None, 0, None, None, None, None,
                                None, None, None, None, 0, None) == _abi.MANO_EINVAL
    out = ctypes.c_void_p()
    uid = ctypes.create_string_buffer(_abi.MANO_COMM_ID_BYTES)
    assert lib.mano_comm_create(0, 2, 2, uid, ctypes.byref(out)) == _abi.MANO_EINVAL
    assert lib.mano_comm_create(0, 1, 0, None, ctypes.byref(out)) == _abi.MANO_EINVAL
    assert lib.mano_comm_destroy(None) == _abi.MANO_OK
    assert lib.mano_gather(None, None, 0, None, None, 0, None) == _abi.MANO_EINVAL
    assert lib.mano_allgather(None, None, 0, None, None) == _abi.MANO_EINVAL
    assert lib.mano_comm_unique_id(None) == _abi.MANO_EINVAL
    # ABI 7: the pre-flight check and the info query refuse a NULL comm too
    assert lib.mano_gather_check(None, None, 0, None, None, 0) == _abi.MANO_EINVAL
    n = ctypes.c_int32(-7)
    assert lib.mano_comm_info(None, ctypes.byref(n), None, None) == _abi.MANO_EINVAL and n.value == -7


def test_makefile_matches_build_flags():
    """`make -C mano-hand_amd` and __graft_entry__.build() compile every source
    with the same per-source flags (the max-ILP scheduler, the MFMA VGPR form)."""
    import re
    import __graft_entry__ as g
    mk = open(os.path.join(REPO, "mano-hand_amd", "Makefile")).read()
    srcs = re.search(r"^SRCS := (.*)$", mk, re.M).group(1).split()
    assert [os.path.basename(x) for x in srcs] == [os.path.basename(x) for x in g.SRCS]
    extra = {m.group(1): m.group(2).split() for m in re.finditer(r"^\$\(OBJDIR\)/(\S+)\.o: EXTRA := (.*)$", mk, re.M)}
    assert extra == {k: v for k, v in g.SRC_FLAGS.items()}


def test_device_status_argument_checks():
    lib = _abi.lib()
    st = ctypes.c_int32(7)
    assert lib.mano_model_device_status(None, ctypes.byref(st), 0) == _abi.MANO_EINVAL
    assert st.value == 7


def test_edevice_maps_to_device_status_error():
    """MANO_EDEVICE (a launch refused while a status bit is set) raises the
    DeviceStatusError the wrappers document, with the bits from the message."""
    import unittest.mock as um
    fake = um.MagicMock()
    fake.mano_last_error.return_value = b"device status 0x1: an earlier launch ..."
    with um.patch.object(_abi, "lib", return_value=fake):
        with pytest.raises(_abi.DeviceStatusError) as ei:
            _abi.check(_abi.MANO_EDEVICE)
    assert ei.value.code == _abi.MANO_EDEVICE and ei.value.status == 1
    assert isinstance(ei.value, _abi.ManoError)


def test_single_process_comm_argument_checks():
    """ABI 6's one-thread-many-devices communicators refuse bad arguments
    before touching RCCL or a GPU."""
    lib = _abi.lib()
    comms = (ctypes.c_void_p * 2)()
    devs = (ctypes.c_int * 2)(0, 0)
    assert lib.mano_comm_create_all(0, devs, comms) == _abi.MANO_EINVAL
    assert lib.mano_comm_create_all(2, None, comms) == _abi.MANO_EINVAL
    assert lib.mano_comm_create_all(2, devs, None) == _abi.MANO_EINVAL
    neg = (ctypes.c_int * 1)(-1)
    assert lib.mano_comm_create_all(1, neg, comms) in (_abi.MANO_EINVAL, _abi.MANO_EHIP)
    assert comms[0] is None


def test_host_block_mapped_is_false_for_pageable_memory():
    """The drop-in's zero-copy guard (hipPointerGetAttributes through the
    runtime libmano_hip.so links) answers False for ordinary pageable host
    memory -- here, with no GPU, for anything -- and never raises."""
    import numpy as np
    from mano_amd import _abi
    a = np.zeros(64, dtype=np.float32)
    assert _abi.host_block_mapped(a.ctypes.data) is False


def test_host_alloc_argument_checks():
    """ABI 5's pinned host allocation: argument checks without a GPU."""
    lib = _abi.lib()
    p = ctypes.c_void_p(1)
    assert lib.mano_host_alloc(0, ctypes.byref(p)) == _abi.MANO_OK and not p.value
    assert lib.mano_host_alloc(16, None) == _abi.MANO_EINVAL
    assert lib.mano_host_free(None) == _abi.MANO_OK


def test_ffi_binding_signatures_match_header():
    """integration/mano_hip_ffi.py (the torch-free binding) declares every C
    function it calls with the header's parameter count, and imports without
    torch and without a GPU (loading the library runs nothing)."""
    import re
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); import mano_hip_ffi as f; "
            "print({n: len(getattr(f._lib, n).argtypes) for n in ('mano_model_create', 'mano_forward', "
            "'mano_alloc', 'mano_free', 'mano_memcpy', 'mano_host_alloc', 'mano_host_free', 'mano_synchronize', "
            "'mano_forward_workspace_bytes', 'mano_model_destroy', 'mano_model_device_status')}); "
            "print('torch' in sys.modules)"
            % os.path.join(REPO, "integration"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    counts, torch_loaded = r.stdout.strip().splitlines()
    assert torch_loaded == "False"
    header = open(os.path.join(REPO, "include", "mano_hip.h")).read()
    for name, n in eval(counts).items():
        m = re.search(r"\b%s\(([^)]*)\)" % name, header)
        assert m, name
        params = [p for p in m.group(1).split(",") if p.strip() and p.strip() != "void"]
        assert len(params) == n, (name, len(params), n)
