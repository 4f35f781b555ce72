#!/bin/bash
# One GPU-box session: smoke, GPU parity tests, bench, rocprofv3 kernel stats.
# Each GPU step has its own time limit; a fault/abort/timeout (rc not 0/1)
# ends the script before any further GPU work.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  tail -5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
step smoke 420 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -m pytest tests -m gpu -q -x
step bench 420 python bench.py --steps 20 --warmup 5
export TMPDIR=/tmp
step rocprof 420 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu
find $OUT/prof -name '*stats*' | head
