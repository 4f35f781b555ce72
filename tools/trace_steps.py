"""The timed steps of a bench run from a rocprofv3 kernel trace: per-launch
durations of articulate_kernel and blend_skin16_kernel and the idle gaps
between consecutive launches, for the last `--steps` (articulate,
blend_skin16) pairs of the trace -- the timed region when the bench ran with
--no-extra --no-check --no-dropin (no launches of these kernels after it).

    python tools/trace_steps.py <dir with *kernel_trace.csv> [--steps 20]

Prints one JSON line: medians / means in microseconds."""
import csv
import json
import os
import statistics
import sys


def main():
    args = sys.argv[1:]
    steps = 20
    if "--steps" in args:
        i = args.index("--steps")
        steps = int(args[i + 1])
        del args[i:i + 2]
    rows = []
    for root, _, files in os.walk(args[0]):
        for fn in files:
            if fn.endswith("kernel_trace.csv"):
                with open(os.path.join(root, fn)) as f:
                    rows += list(csv.DictReader(f))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    seq = []
    for r in rows:
        name = r["Kernel_Name"]
        kind = "articulate" if "articulate_kernel" in name else "blend_skin" if "blend_skin16_kernel" in name else None
        seq.append((kind, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    # last `steps` pairs (articulate followed by blend_skin16)
    idx = [i for i in range(len(seq) - 1) if seq[i][0] == "articulate" and seq[i + 1][0] == "blend_skin"]
    idx = idx[-steps:]
    art = [(seq[i][2] - seq[i][1]) / 1e3 for i in idx]
    bs = [(seq[i + 1][2] - seq[i + 1][1]) / 1e3 for i in idx]
    gap_a = [(seq[i][1] - seq[i - 1][2]) / 1e3 for i in idx if i > 0]       # before articulate
    gap_b = [(seq[i + 1][1] - seq[i][2]) / 1e3 for i in idx]               # articulate -> blend_skin16
    span = (seq[idx[-1] + 1][2] - seq[idx[0]][1]) / 1e3 if idx else None
    med = lambda x: statistics.median(x) if x else None  # noqa: E731
    print(json.dumps({"pairs": len(idx), "articulate_us": {"median": med(art), "mean": statistics.fmean(art) if art else None,
                                                          "max": max(art) if art else None},
                      "blend_skin_us": {"median": med(bs), "mean": statistics.fmean(bs) if bs else None},
                      "gap_before_articulate_us": {"median": med(gap_a), "max": max(gap_a) if gap_a else None},
                      "gap_articulate_to_blend_us": {"median": med(gap_b), "max": max(gap_b) if gap_b else None},
                      "span_us": span, "us_per_step": span / len(idx) if idx else None}))


if __name__ == "__main__":
    main()
