"""Host-side model packing (mano-hand_amd/csrc/mano_pack.cpp) under AddressSanitizer
and UBSan, on the CPU (host ASan on the C-ABI packing code).

The packing is plain C++ (no HIP), so g++ builds it together with
tests/native/pack_check.cpp, which decodes every fragment layout of packed
random models (the MANO mesh and small meshes covering the tail-group cases)
back to the dump-layout arrays and checks the argument errors."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "mano-hand_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_pack_model_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "pack_check")
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-Wall", "-I", CSRC,
           os.path.join(REPO, "tests", "native", "pack_check.cpp"), os.path.join(CSRC, "mano_pack.cpp"),
           "-o", exe]
    b = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "V= 778 ok" in r.stdout and "argument errors ok" in r.stdout
