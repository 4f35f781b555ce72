"""Disassemble every gfx950 code object of the built library (tools/isa_scan.py)
and count the instructions the design keeps out of it: packed
fp32 VALU and scalar-cache stores; record isa_scan's check of skin_pair's
hand-counted vmcnt protocol.  Writes <lib>.codegen.json next to the library; run by
__graft_entry__.build() and `make`, read by tests/test_codegen.py.

    python tools/codegen_report.py [path/to/libmano_hip.so]

(Disassembly runs here, at build time, in a process without the HIP runtime:
child processes of a process that has loaded the runtime make it crash later
in this container.)"""
import hashlib
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_scan  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "mano-hand_amd", "mano_amd", "libmano_hip.so")
WATCH = {
    "packed_fp32": re.compile(r"\bv_pk_(fma|mul|add)_f32\b"),
    "scalar_store": re.compile(r"\b(s_store_dword\w*|s_buffer_store\w*|s_scratch_store\w*|s_dcache_wb\w*|s_dcache_discard\w*|s_atomic_\w*|s_buffer_atomic_\w*)\b"),
}


def main(lib=LIB):
    asm, scan = isa_scan.scan(lib)
    report = {
        "lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(),
        "mfma": {m: n for m, n in sorted(
            {op: len(re.findall(rf"\b{op}\b", asm)) for op in set(re.findall(r"\bv_mfma_\w+", asm))}.items())},
        "counts": {k: len(rx.findall(asm)) for k, rx in WATCH.items()},
        "examples": {k: [l.strip() for l in asm.splitlines() if rx.search(l)][:5] for k, rx in WATCH.items()},
        "skin_pair_vmcnt": scan["skin_pair_vmcnt"],
        "repeated_store_data": scan["repeated_store_data"],
    }
    with open(lib + ".codegen.json", "w") as f:
        json.dump(report, f, indent=1)
    print(json.dumps({k: report[k] for k in ("mfma", "counts")} |
                     {"skin_pair_vmcnt_ok": all(v["ok"] for v in scan["skin_pair_vmcnt"].values()),
                      "repeated_store_data": len(scan["repeated_store_data"])}))


if __name__ == "__main__":
    main(*sys.argv[1:])
