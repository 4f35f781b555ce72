#!/bin/bash
# rocprofv3 evidence per workload: kernel-trace stats and separate FETCH_SIZE /
# WRITE_SIZE passes of bench.py at the C2 / C5 / C3 sizes (one GPU).
# Usage (GPU box): TAG=r02 bash tools/pmc_workloads.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${TAG:-r02}
mkdir -p $OUT
run() {  # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.log"; exit $rc; fi
}
run stats_C2 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_C2 -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu --no-dropin --no-check --no-live-pmc
run stats_C5 300 rocprofv3 --kernel-trace --stats -d $OUT/stats_C5 -o run --output-format csv -- python bench.py --workload C5 --steps 20 --warmup 5 --no-cpu --no-dropin --no-check --no-live-pmc --no-extra
for W in C2:65536 C5:1048576 C3:2097152; do
  name=${W%%:*}; batch=${W#*:}
  extra="--no-extra"; [ "$name" = C2 ] && extra=""
  run fetch_$name 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/$batch/fetch -o p --output-format csv -- python bench.py --workload $name --steps 3 --warmup 1 --ramp-seconds 0 --no-cpu --no-dropin --no-check --no-live-pmc $extra
  run write_$name 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/$batch/write -o p --output-format csv -- python bench.py --workload $name --steps 3 --warmup 1 --ramp-seconds 0 --no-cpu --no-dropin --no-check --no-live-pmc $extra
done
# MFMA busy / wave states / clock of C2's kernels: SQ + GRBM counters with the
# kernel trace (durations) in one pass (no system/runtime trace with --pmc)
run sq_C2 200 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $OUT/65536/sq -o p --output-format csv -- python bench.py --steps 3 --warmup 1 --ramp-seconds 0.5 --no-cpu --no-dropin --no-check --no-live-pmc
python tools/pmc_traffic.py $OUT $OUT/pmc_traffic.json
