#!/bin/bash
# HBM bytes per launch of every kernel of one forward path, from two separate
# rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE: the counter budget of one
# pass, MI355X_MICROARCH.md) over tools/debug/run_path.py.
#   bash tools/pmc_path.sh unfused skin_b2b staged rest_verts
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmc_path}
mkdir -p $OUT
for p in "$@"; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 120 rocprofv3 --pmc $c -d $OUT/$p/$c -o p --output-format csv -- python tools/debug/run_path.py $p 20 > $OUT/$p.$c.log 2>&1 || { echo "$p $c failed"; tail -5 $OUT/$p.$c.log; exit 1; }
  done
done
python3 - "$OUT" "$@" <<'PY'
import csv, glob, json, os, sys, collections
out = sys.argv[1]
res = {}
for p in sys.argv[2:]:
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        for f in glob.glob(f"{out}/{p}/{c}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if r["Counter_Name"] != c:
                    continue
                # strip the namespace first: "(anonymous namespace)" holds a "("
                k = r["Kernel_Name"].replace("void ", "").replace("mano::(anonymous namespace)::", "").split("(")[0]
                acc[k][c].append(float(r["Counter_Value"]))
    res[p] = {k: {"read_bytes": 2 * 1024 * sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"]),
                  "write_bytes": 1024 * sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"]),
                  "launches": len(d["WRITE_SIZE"])}
              for k, d in acc.items() if d["FETCH_SIZE"] and d["WRITE_SIZE"]}
json.dump(res, open(f"{out}/pmc_path.json", "w"), indent=1)
for p, ks in res.items():
    for k, v in ks.items():
        print(f"{p:11s} {k[:60]:60s} read {v['read_bytes']/1e6:8.1f} MB  write {v['write_bytes']/1e6:8.1f} MB")
PY
