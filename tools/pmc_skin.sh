#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_skin
mkdir -p $OUT
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS"; do
  tag=$(echo $set | cut -d' ' -f1)
  timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $OUT/$tag -o run -- ./tools/microbench/skin_variants > $OUT/$tag.log 2>&1
  rc=$?; echo "$tag rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/$tag.log; fi
done
