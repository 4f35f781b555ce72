"""Merge per-workload rocprofv3 --pmc summaries into profiles/pmc_traffic.json.

    python tools/pmc_traffic.py gpurun_out/pmc_r02 [out.json]

Expects <dir>/<batch>/{fetch,write}/... from tools/pmc_workloads.sh (one
FETCH_SIZE and one WRITE_SIZE pass per workload batch, separate runs), and
writes {"kernels": {key: [{"batch": B, "hbm_bytes_per_launch": ...}, ...]}}
-- the form bench.py's load_traffic reads (an entry per measured batch)."""
import io
import json
import os
import sys
from contextlib import redirect_stdout

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import summarize_pmc  # noqa: E402


def main(root, dst):
    merged = {"method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of "
                        "bench.py --workload W --steps 3; hbm_read = 2 x FETCH_SIZE x 1024 (gfx950 "
                        "counts half of a wide coalesced read, MI355X_MICROARCH.md), hbm_write = "
                        "WRITE_SIZE x 1024, averaged over the kernel's dispatches",
              "kernels": {}}
    for name in sorted(os.listdir(root)):
        if not name.isdigit():
            continue
        buf = io.StringIO()
        with redirect_stdout(buf):
            summarize_pmc.main(os.path.join(root, name), int(name))
        res = json.loads(buf.getvalue().strip().splitlines()[-1])
        for k, v in res["kernels"].items():
            merged["kernels"].setdefault(k, []).append(dict(v, batch=int(name)))
    with open(dst, "w") as f:
        json.dump(merged, f, indent=1)
    for k, ents in merged["kernels"].items():
        print(k, [(e["batch"], round(e["hbm_bytes_per_launch"] / e["batch"])) for e in ents], "B/hand")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json"))
