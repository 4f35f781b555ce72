#!/bin/bash
# f16x3 iteration: the fused-vs-standalone LBS check, every GPU test, then both
# benches (no CPU baseline).  Each GPU step has its own time limit; a fault,
# abort or timeout (rc not 0/1) ends the script before any further GPU work.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/h3
mkdir -p $OUT
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -${TAILN:-6} "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
step variants 240 python -u tools/debug/h3_fused_variants.py
TAILN=12 step pytest 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench_h3 300 python bench.py --no-cpu --precision f16x3
step bench_fp32 300 python bench.py --no-cpu
