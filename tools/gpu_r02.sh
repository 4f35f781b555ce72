#!/bin/bash
# Round-2 GPU session: smoke, the GPU suite, the bench at the driver's flags and
# at each workload, the 2-rank launcher rehearsal, rocprofv3 kernel stats.
# Each GPU step has its own time limit; a fault/abort/timeout (rc not 0/1)
# ends the script before any further GPU work.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r02}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  tail -3 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread
step bench_driver 300 python bench.py --steps 20 --warmup 5
step bench_c5 300 python bench.py --workload C5 --steps 50 --warmup 5 --no-cpu --no-extra
step bench_c3 300 python bench.py --workload C3 --steps 30 --warmup 3 --no-cpu --no-extra
step bench_c4 300 python bench.py --workload C4 --steps 50 --warmup 5 --no-cpu --no-extra
step bench_dp2 300 python bench.py --gpus 2 --backend gloo --steps 20 --warmup 5 --no-cpu --no-extra
step rocprof 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu
find $OUT/prof -name '*stats*'
