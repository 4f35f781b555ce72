"""Per-launch durations of the MANO kernels from a rocprofv3 kernel-trace CSV.

    python tools/trace_durations.py <run_kernel_trace.csv> [name-substring ...]
"""
import csv
import sys


def main():
    path = sys.argv[1]
    keys = sys.argv[2:] or ["mano::"]
    with open(path) as f:
        rows = list(csv.DictReader(f))
    for r in rows:
        name = r["Kernel_Name"]
        if not any(k in name for k in keys):
            continue
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        short = name.replace("mano::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        print(f"{short[:40]:40s} grid={r.get('Grid_Size_X', ''):>7s} us={d:.1f} "
              f"vgpr={r.get('VGPR_Count', '')} agpr={r.get('Accum_VGPR_Count', '')} "
              f"sgpr={r.get('SGPR_Count', '')} scratch={r.get('Scratch_Size', '')}")


if __name__ == "__main__":
    main()
