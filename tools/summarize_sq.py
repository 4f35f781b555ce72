"""Per-kernel MFMA busy fraction, wave-state split and effective clock from a
rocprofv3 `--kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES
SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE`
pass (tools/pmc_workloads.sh):

    python tools/summarize_sq.py <pass dir> [out.json]

clock = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs) / kernel duration
(MI355X_MICROARCH.md 'DVFS give-back'; reads high below ~0.3 ms);
MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8)."""
import collections
import csv
import glob
import json
import sys

KERNELS = {"blend_skin16_kernel<": "blend_skin", "articulate_kernel<": "articulate", "skin_pair_kernel<": "skin",
           "skin_span_kernel<": "skin", "blend_kernel(": "blend", "blend_skin_h3_kernel<": "blend_skin_h3",
           "skin_span_h3_kernel<": "skin_h3"}


def short(name):
    if "::skin_pair_kernel<" in name and ", true>" in name.split("(")[1 if name.startswith("void") else 0]:
        return "skin_h3"  # skin_pair_kernel<kTrans, kH3 = true>: the f16x3 standalone LBS
    for k, v in KERNELS.items():
        if "::" + k in name:
            return v
    return None


def main(d, dst=None):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k:
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    dur = collections.defaultdict(list)
    for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k:
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    out = {}
    for k, cs in sorted(acc.items()):
        a = {c: sum(v) / len(v) for c, v in cs.items()}
        t = sum(dur[k]) / len(dur[k])
        cyc = a["GRBM_GUI_ACTIVE"] / 8
        wc = a["SQ_WAVE_CYCLES"]
        out[k] = {"dispatches": len(cs["GRBM_GUI_ACTIVE"]), "ms": t * 1e3, "clock_ghz": cyc / t / 1e9,
                  "mfma_busy": a["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / cyc,
                  "wave_issue_wait": a["SQ_WAIT_INST_ANY"] / wc, "wave_waitcnt_barrier": a["SQ_WAIT_ANY"] / wc,
                  "wave_active": a["SQ_ACTIVE_INST_ANY"] / wc}
        print(k, {x: round(y, 4) for x, y in out[k].items()})
    if dst:
        with open(dst, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
