#!/bin/bash
# rocprofv3 evidence for one round: kernel-trace stats of the default bench and
# separate PMC passes (FETCH_SIZE / WRITE_SIZE / SQ / L2).  The default bench
# times the fused forward and, after its timed region, the staged and unfused
# kernels, so one run covers every kernel.
# Usage: bash tools/profile_round.sh r01
set -u
TAG=${1:-r01}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
run() {  # name timeout args...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.log"; exit $rc; fi
}
# The default warmup (300 launches) so the averages are steady-clock ones, as in bench.py.
run stats 400 rocprofv3 --kernel-trace --stats -d $OUT/stats -o bench --output-format csv -- python bench.py --no-cpu
B="python bench.py --steps 5 --warmup 2 --no-cpu"
run fetch 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o p --output-format csv -- $B
run write 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o p --output-format csv -- $B
run sq 300 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES -d $OUT/sq -o p --output-format csv -- $B
run l2 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT TCC_HIT_sum TCC_MISS_sum -d $OUT/l2 -o p --output-format csv -- $B
run waits 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS -d $OUT/waits -o p --output-format csv -- $B
python tools/summarize_pmc.py $OUT > $OUT/summary.txt 2>&1; echo summarize rc=$?
head -80 $OUT/summary.txt
