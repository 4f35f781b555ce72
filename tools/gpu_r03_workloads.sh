#!/bin/bash
# Round-3 evidence per BASELINE config on one GPU: the bench at C5 / C3 / C4
# (the C4 shard with the gather path at N = 1), the 2-rank gloo rehearsal of
# the C4 gather, then the per-workload rocprofv3 stats and PMC traffic passes
# (tools/pmc_workloads.sh).  Each GPU step time-limited; stop on a fault.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03w}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  tail -2 "$OUT/$name.log" | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
step bench_c5 300 python bench.py --workload C5 --steps 50 --warmup 5 --no-cpu --no-extra
step bench_c3 300 python bench.py --workload C3 --steps 30 --warmup 3 --no-cpu --no-extra
step bench_c4 300 python bench.py --workload C4 --steps 50 --warmup 5 --no-cpu --no-extra
step bench_c4_dp2 300 python bench.py --gpus 2 --backend gloo --workload C4 --batch 65536 --steps 10 --warmup 3 --no-cpu --no-extra
step pmc 900 env TAG=${TAG:-r03w} bash tools/pmc_workloads.sh
