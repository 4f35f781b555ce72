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


def test_no_slp_vectorize_flag_on_every_build():
    """The f16x3 kernels' correctness rests on -fno-slp-vectorize (no packed
    fp32 beside their MFMAs; mano_kernels_h3.hip header): both build recipes
    -- __graft_entry__.build() and the Makefile -- pass it to every source."""
    import re
    import __graft_entry__ as g
    assert "-fno-slp-vectorize" in g.FLAGS
    mk = open(os.path.join(REPO, "mano-hand_amd", "Makefile")).read()
    flags = re.search(r"^CXXFLAGS \?= (.*)$", mk, re.M).group(1).split()
    assert "-fno-slp-vectorize" in flags


def test_kernels_present(report):
    assert report["mfma"].get("v_mfma_f32_16x16x4_f32", 0) > 0       # fp32 kernels
    assert report["mfma"].get("v_mfma_f32_16x16x32_f16", 0) > 0      # f16x3 kernels


def test_no_packed_fp32_valu(report):
    assert report["counts"]["packed_fp32"] == 0, report["examples"]["packed_fp32"]


def test_no_scalar_stores(report):
    assert report["counts"]["scalar_store"] == 0, report["examples"]["scalar_store"]


def test_skin_pair_vmcnt_protocol(report):
    """skin_pair's memory wave waits with a hand-counted s_waitcnt vmcnt(N):
    on every control-flow path into that wait the disassembly must end with
    the awaited unit's DMA group, >= 3 stores, then exactly one DMA group
    (tools/isa_scan.py), in all eight instantiations."""
    pairs = report["skin_pair_vmcnt"]
    assert len(pairs) == 8, sorted(pairs)  # fp32 x trans x (plain, aligned, in-place) units + f16x3 x trans
    for name, r in pairs.items():
        assert r["waits"] >= 1 and r["ok"], (name, r)


def test_no_repeated_store_data(report):
    """tools/isa_scan.py rule 3: no run of stores of one unchanged data
    register (the ext_vector bit_cast pitfall's shape) in any kernel."""
    assert report["repeated_store_data"] == {}, report["repeated_store_data"]


def test_repeated_store_rule_catches_the_bitcast_pitfall(tmp_path):
    """The rule on a two-kernel fixture compiled here: the pitfall form
    (__builtin_bit_cast of an ext_vector element: element 0 stored for every
    row) is flagged, the product's form (a scalar copy first) is not."""
    import subprocess
    hipcc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not installed")
    out = tmp_path / "pitfall.s"
    r = subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "--cuda-device-only", "-S", "-o", str(out),
                        os.path.join(REPO, "tests", "native", "bitcast_pitfall.hip")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    isa_scan = _tools()
    flagged = isa_scan.scan_repeated_stores(out.read_text())
    assert any("bug_kernel" in k for k in flagged), flagged
    assert not any("ok_kernel" in k for k in flagged), flagged


def _tools():
    import sys
    p = os.path.join(REPO, "tools")
    if p not in sys.path:
        sys.path.insert(0, p)
    import isa_scan
    return isa_scan


def _prog(ops):
    """A straight-line instruction list for isa_scan.check_vmcnt_protocol."""
    code = {"dma": ("buffer_load_dwordx4", "v8, s[0:3], 0 offen lds"),
            "st": ("buffer_store_dwordx4", "v[0:3], v4, s[0:3], 0 offen"),
            "wait": ("s_waitcnt", "vmcnt(10)"), "end": ("s_endpgm", "")}
    return [(4 * i, *code[o], None) for i, o in enumerate(ops)]


def test_vmcnt_checker_catches_reordered_ops():
    """The protocol checker itself: the kernel's order passes; a DMA moved
    ahead of a store, a missing store or a split group fails."""
    s = _tools()
    dma7 = ["dma"] * 7
    good = dma7 + ["st"] * 3 + dma7 + ["wait", "end"]
    assert s.check_vmcnt_protocol(_prog(good), 7, 10) == (1, [])
    bad_order = dma7 + ["st"] * 2 + ["dma", "st"] + ["dma"] * 6 + ["wait", "end"]
    bad_missing = dma7 + ["st"] * 2 + dma7 + ["wait", "end"]
    bad_short = dma7 + ["st"] * 3 + ["dma"] * 6 + ["wait", "end"]
    for prog in (bad_order, bad_missing, bad_short):
        n, fails = s.check_vmcnt_protocol(_prog(prog), 7, 10)
        assert n == 1 and fails, prog


def test_product_build_sets_no_diagnostic_switch():
    """Every MANO_* knob the kernel sources read is guarded by csrc/mano_diag.h
    (#error unless MANO_DIAGNOSTIC_BUILD), and the product build flags
    (__graft_entry__.py, the Makefile) define none of them."""
    import re
    import subprocess
    import __graft_entry__ as g
    csrc = os.path.join(REPO, "mano-hand_amd", "csrc")
    knobs = set()
    for fn in os.listdir(csrc):
        knobs |= set(re.findall(r"#ifndef (MANO_[A-Z0-9_]+)", open(os.path.join(csrc, fn)).read()))
    knobs -= {"MANO_HIP_H"}
    guard = open(os.path.join(csrc, "mano_diag.h")).read()
    listed = set(re.findall(r"defined\((MANO_[A-Z0-9_]+)\)", guard)) - {"MANO_DIAGNOSTIC_BUILD"}
    assert knobs <= listed, sorted(knobs - listed)
    flags = " ".join(g.FLAGS + [x for v in g.SRC_FLAGS.values() for x in v])
    mk = open(os.path.join(REPO, "mano-hand_amd", "Makefile")).read()
    assert "-DMANO" not in flags and "-DMANO" not in mk
    # the guard fires on a knob and stays quiet without one / in a tools build
    hdr = os.path.join(csrc, "mano_layout.h")
    run = lambda *d: subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-x", "c++", *d, hdr],  # noqa: E731
                                    capture_output=True, text=True)
    assert run().returncode == 0
    r = run("-DMANO_BS_ABLATE=1")
    assert r.returncode != 0 and "diagnostic" in r.stderr
    assert run("-DMANO_BS_ABLATE=1", "-DMANO_DIAGNOSTIC_BUILD=1").returncode == 0
    with pytest.raises(ValueError):
        g.build_library(g.LIB, ["-DMANO_BS_ABLATE=1"])


def _prog_insts(lines):
    """(addr, mnemonic, operands, branch target) tuples, 4 bytes apart; a
    target is given as the index of the instruction it jumps to."""
    out = []
    for k, (mn, ops, tgt) in enumerate(lines):
        out.append((4 * k, mn, ops, None if tgt is None else 4 * tgt))
    return out


def test_vmcnt_scan_follows_the_structurizer_flow_variable():
    """tools/isa_scan.py on the shape the compiler gives a uniform if / else
    (skin_pair's in-place cold / hot spans): arm A guarded by an SCC branch
    clears a flow variable, arm B is skipped through `s_andn2_b64 vcc, exec,
    flow` -- every followed path runs exactly one arm, so the 2-op DMA group
    checks out.  Without the flow variable (a genuine both-arms path) the
    same program fails."""
    isa_scan = _tools()
    dma, st = ("buffer_load_dwordx4", "v1, s[0:3], 0 offen lds", None), ("buffer_store_dwordx4", "v[0:3], v4, s[0:3], 0 offen", None)
    body = [
        dma, dma,                                   # 0-1: unit k's DMA group (2 ops)
        st, st, st,                                 # 2-4: stores
        ("s_mov_b64", "s[44:45], -1", None),        # 5: flow = -1
        ("s_cbranch_scc1", "1", 9),                 # 6: cold -> skip arm A
        dma, dma,                                   # 7-8: arm A (default policy)
        ("s_mov_b64", "s[44:45], 0", None),         # 9: (A ran) flow = 0   [target of 6 is 10 below]
        ("s_andn2_b64", "vcc, exec, s[44:45]", None),
        ("s_cbranch_vccnz", "1", 14),               # 11: A ran -> skip arm B
        ("buffer_load_dwordx4", "v1, s[0:3], 0 offen nt lds", None),
        ("buffer_load_dwordx4", "v1, s[0:3], 0 offen nt lds", None),
        ("s_waitcnt", "vmcnt(5)", None),            # 14
        ("s_endpgm", "", None),
    ]
    body[6] = ("s_cbranch_scc1", "1", 10)
    n, fails = isa_scan.check_vmcnt_protocol(_prog_insts(body), 2, 5, n_stores=3)
    assert n == 1 and fails == [], fails
    broken = [l for k, l in enumerate(body) if k not in (5, 9)]   # no flow variable: vcc unknown
    for k, l in enumerate(broken):
        if l[0].startswith("s_cbranch") and l[2] is not None:
            broken[k] = (l[0], l[1], l[2] - (1 if l[2] > 5 else 0) - (1 if l[2] > 9 else 0))
    n, fails = isa_scan.check_vmcnt_protocol(_prog_insts(broken), 2, 5, n_stores=3)
    assert n == 1 and fails, "a path through both arms must fail"
