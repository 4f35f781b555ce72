"""Code-generation guards on the built gfx950 library (CPU only: the code
object is disassembled, nothing runs).

Packed fp32 VALU (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32) is kept out of
every kernel: with it, blend_skin_h3 returned wrong verts in lanes 48-63 of
some tiles ("Packed fp32 VALU is a correctness hazard"), and it
is the slower form beside the MFMAs.  The library is built with
-fno-slp-vectorize; this test fails if any packed fp32 op comes back.
"""
import os
import shutil
import subprocess

import pytest

from conftest import REPO

LIB = os.path.join(REPO, "mano-hand_amd", "mano_amd", "libmano_hip.so")
LLVM = "/opt/rocm/llvm/bin"


def _disassemble(tmp_path):
    if not os.path.exists(LIB):
        pytest.skip("library not built")
    for tool in ("objcopy",):
        if shutil.which(tool) is None:
            pytest.skip(f"{tool} missing")
    bundler = os.path.join(LLVM, "clang-offload-bundler")
    objdump = os.path.join(LLVM, "llvm-objdump")
    if not (os.path.exists(bundler) and os.path.exists(objdump)):
        pytest.skip("ROCm LLVM tools missing")
    fat = tmp_path / "fatbin.bin"
    subprocess.run(["objcopy", f"--dump-section=.hip_fatbin={fat}", LIB], check=True)
    # One offload bundle per translation unit, concatenated (aligned) in the section.
    data = fat.read_bytes()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = []
    i = data.find(magic)
    while i >= 0:
        starts.append(i)
        i = data.find(magic, i + 1)
    out = []
    for k, a in enumerate(starts):
        b = starts[k + 1] if k + 1 < len(starts) else len(data)
        part, co = tmp_path / f"bundle{k}.bin", tmp_path / f"gfx950_{k}.co"
        part.write_bytes(data[a:b])
        subprocess.run([bundler, "--unbundle", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        f"--input={part}", f"--output={co}"], check=True)
        out.append(subprocess.run([objdump, "-d", "--mcpu=gfx950", str(co)], check=True,
                                  capture_output=True, text=True).stdout)
    return "\n".join(out)


def test_no_packed_fp32_valu(tmp_path):
    asm = _disassemble(tmp_path)
    assert "v_mfma_f32_16x16x4" in asm and "v_mfma_f32_16x16x32_f16" in asm  # the kernels are there
    packed = [l for l in asm.splitlines()
              if any(op in l for op in ("v_pk_fma_f32", "v_pk_mul_f32", "v_pk_add_f32"))]
    assert not packed, f"{len(packed)} packed fp32 instructions, e.g. {packed[:3]}"


def test_no_scalar_stores(tmp_path):
    """No write through the scalar data cache anywhere (s_store / s_dcache_wb)."""
    asm = _disassemble(tmp_path)
    bad = [l for l in asm.splitlines() if "s_store_dword" in l or "s_dcache_wb" in l
           or "s_buffer_store" in l or "s_scratch_store" in l]
    assert not bad, bad[:3]
