#!/bin/bash
# A/B timing of library variants, interleaved twice.
#   bash tools/gpu_ab_skin.sh base p1 ...          standalone LBS (time_skin.py)
#   TOOL=time_forward bash tools/gpu_ab_skin.sh ... fused forward kernel
# (libraries mano-hand_amd/mano_amd/libmano_hip_<name>.so, built beforehand).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
TOOL=${TOOL:-time_skin}
OUT=gpurun_out/ab_$TOOL; mkdir -p $OUT
for r in 1 2; do for v in "$@"; do
  timeout -k 10 120 python -u tools/debug/$TOOL.py libmano_hip_$v.so >> $OUT/t.log 2>&1 || { echo fail $v; tail -5 $OUT/t.log; exit 3; }
done; done
grep libmano $OUT/t.log
