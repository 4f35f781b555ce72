"""Summarise a tools/profile_round.sh directory into per-kernel averages.

HBM traffic per launch follows /opt/skills/guides/MI355X_MICROARCH.md §HBM:
FETCH_SIZE (KB) reads exactly half the bytes of a wide coalesced stream on
gfx950, so hbm_read = 2 * FETCH_SIZE * 1024 (an upper estimate for narrower
accesses); hbm_write = WRITE_SIZE * 1024.  Writes `pmc_traffic.json`-style
JSON on stdout's last line and a readable table before it.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

# demangled-name prefix -> bench.py kernel key
KERNELS = {"blend_skin16_kernel<": "blend_skin", "blend_kernel(": "blend", "skin_span_kernel<": "skin", "skin_pair_kernel<": "skin",
           "articulate_kernel<": "articulate", "blend_skin_h3_kernel<": "blend_skin_h3",
           "skin_span_h3_kernel<": "skin_h3"}
# FETCH_SIZE correction (MI355X_MICROARCH.md §HBM): on gfx950 the counter
# reports half the bytes of wide coalesced streams.  Measured here it is x2 for
# every kernel of this path, dwordx3 streams included: skin16 raw 350.6 MB vs
# 662 MB algorithmic reads, articulate raw 7.7 MB vs 15.2 MB (65,536 hands).
FETCH_FACTOR = {"blend_skin": 2.0, "blend": 2.0, "skin": 2.0, "articulate": 2.0,
                "blend_skin_h3": 2.0, "skin_h3": 2.0}


def short(name):
    if "::skin_pair_kernel<" in name and ", true>" in name.split("(")[1 if name.startswith("void") else 0]:
        return "skin_h3"  # skin_pair_kernel<kTrans, kH3 = true>: the f16x3 standalone LBS
    for k, v in KERNELS.items():
        if "::" + k in name:
            return v
    return None


def main(d, batch=65536):
    acc = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> per-dispatch values
    for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k is not None:
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {"batch": batch, "kernels": {}}
    for k, cs in sorted(acc.items()):
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        print(f"{k:12s}")
        for c, v in sorted(avg.items()):
            print(f"    {c:32s} {v:.6g}")
        if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
            rd = FETCH_FACTOR[k] * avg["FETCH_SIZE"] * 1024
            wr = avg["WRITE_SIZE"] * 1024
            print(f"    -> hbm read {rd/1e6:.1f} MB ({FETCH_FACTOR[k]:g}x FETCH_SIZE), write {wr/1e6:.1f} MB per launch")
            out["kernels"][k] = {"hbm_bytes_per_launch": rd + wr, "hbm_read_bytes": rd,
                                 "hbm_write_bytes": wr, "fetch_size_kb": avg["FETCH_SIZE"],
                                 "write_size_kb": avg["WRITE_SIZE"],
                                 "fetch_factor": FETCH_FACTOR[k]}
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 65536)
