#!/bin/bash
# A/B timing of standalone-LBS library variants (tools/debug/time_skin.py),
# interleaved twice.  Usage: bash tools/gpu_ab_skin.sh base p1 ...
# (libraries mano-hand_amd/mano_amd/libmano_hip_<name>.so, built beforehand).
set -u
cd "${GRAFT_REPO_ROOT:-.}"
OUT=gpurun_out/abskin; mkdir -p $OUT
for r in 1 2; do for v in "$@"; do
  timeout -k 10 120 python -u tools/debug/time_skin.py libmano_hip_$v.so >> $OUT/t.log 2>&1 || { echo fail $v; tail -5 $OUT/t.log; exit 3; }
done; done
grep skin $OUT/t.log
