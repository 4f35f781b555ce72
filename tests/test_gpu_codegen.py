"""The code object the GPU tests run: no packed fp32 VALU, no repeated store
data, and skin_pair's
hand-counted vmcnt protocol intact (tools/isa_scan.py).

The disassembly is taken when this module is imported -- at collection,
before any test initialises HIP -- in a child process, of the library file
`mano_amd._abi` loads; the test then checks that the library this process
actually mapped is that same file with the same bytes.  (The CPU twin,
tests/test_codegen.py, reads the report written at build time; this one
re-derives it on the GPU box from the library there.)"""
import hashlib
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu

_LIB = os.path.join(REPO, "mano-hand_amd", "mano_amd", "libmano_hip.so")


def _scan():
    if not os.path.exists(_LIB):
        return None, None, "library not built"
    sha = hashlib.sha256(open(_LIB, "rb").read()).hexdigest()
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "isa_scan.py"), "--json", _LIB],
                       capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        return sha, None, r.stderr[-2000:]
    return sha, json.loads(r.stdout.strip().splitlines()[-1]), None


_SHA, _REPORT, _ERR = _scan()


def test_scanned_library_is_the_loaded_one():
    from mano_amd import _abi
    assert _REPORT is not None, _ERR
    lib = _abi.lib()
    assert lib.mano_abi_version() >= 3
    maps = open("/proc/self/maps").read()
    mapped = {l.split()[-1] for l in maps.splitlines() if l.endswith("libmano_hip.so")}
    assert mapped == {os.path.realpath(_abi.LIB_PATH)}, mapped
    assert os.path.realpath(_abi.LIB_PATH) == os.path.realpath(_LIB)
    assert hashlib.sha256(open(_LIB, "rb").read()).hexdigest() == _SHA


def test_no_packed_fp32_in_loaded_library():
    assert _REPORT is not None, _ERR
    assert _REPORT["packed_fp32"] == 0, _REPORT["packed_fp32_examples"]
    assert _REPORT["mfma"].get("v_mfma_f32_16x16x4_f32", 0) > 0


def test_skin_pair_vmcnt_protocol_in_loaded_library():
    assert _REPORT is not None, _ERR
    pairs = _REPORT["skin_pair_vmcnt"]
    assert len(pairs) == 8  # fp32 x trans x (plain, aligned, in-place) units + f16x3 x trans
    for name, r in pairs.items():
        assert r["ok"], (name, r)


def test_no_repeated_store_data_in_loaded_library():
    """isa_scan rule 3 (the ext_vector bit_cast pitfall's shape) on the
    library the GPU tests map."""
    assert _REPORT is not None, _ERR
    assert _REPORT["repeated_store_data"] == {}, _REPORT["repeated_store_data"]
