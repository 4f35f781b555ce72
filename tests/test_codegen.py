"""Code-generation guards on the built gfx950 library (CPU only).

Packed fp32 VALU (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32) is kept out of
every kernel: with it, blend_skin_h3 returned wrong verts in lanes 48-63 of
some tiles ("Packed fp32 VALU is a correctness hazard"), and it
is the slower form beside the MFMAs; the library is built with
-fno-slp-vectorize.  Nothing may write through the scalar data cache.

The disassembly is made at build time (tools/codegen_report.py, run by
__graft_entry__.build() and make) and read here, for the library on disk.
"""
import hashlib
import json
import os

import pytest

from conftest import REPO

LIB = os.path.join(REPO, "mano-hand_amd", "mano_amd", "libmano_hip.so")


@pytest.fixture(scope="module")
def report():
    if not os.path.exists(LIB):
        pytest.skip("library not built")
    path = LIB + ".codegen.json"
    assert os.path.exists(path), "no codegen report: build with __graft_entry__.build() or make"
    rep = json.load(open(path))
    assert rep["lib_sha256"] == hashlib.sha256(open(LIB, "rb").read()).hexdigest(), \
        "codegen report is stale: rebuild"
    return rep


def test_kernels_present(report):
    assert report["mfma"].get("v_mfma_f32_16x16x4_f32", 0) > 0       # fp32 kernels
    assert report["mfma"].get("v_mfma_f32_16x16x32_f16", 0) > 0      # f16x3 kernels


def test_no_packed_fp32_valu(report):
    assert report["counts"]["packed_fp32"] == 0, report["examples"]["packed_fp32"]


def test_no_scalar_stores(report):
    assert report["counts"]["scalar_store"] == 0, report["examples"]["scalar_store"]
