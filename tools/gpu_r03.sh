#!/bin/bash
# Round-3 GPU evidence: the GPU suite, smoke, the default bench (CPU baseline,
# live PMC traffic, correctness leg) and the rocprofv3 kernel-trace stats of
# the same bench command.  Every GPU step time-limited; stop on a fault.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  tail -3 "$OUT/$name.log" | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
if [ -z "${SKIP_TESTS:-}" ]; then
  step pytest_gpu 1000 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread ${PYTEST_ARGS:-}
fi
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python bench.py --steps 20 --warmup 5
step stats 400 rocprofv3 --kernel-trace --stats -d $OUT/stats -o bench --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu --no-live-pmc --no-dropin
if [ -n "${EXTRA:-}" ]; then step extra 600 bash -c "$EXTRA"; fi
