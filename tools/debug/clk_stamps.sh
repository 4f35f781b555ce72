#!/bin/bash
# blend_skin16 in-kernel clock and per-SIMD exit spread (MANO_BS_STAMP builds;
# tools/debug/bs_stamps.py) after WARM back-to-back launches.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-clk}; mkdir -p $OUT
for lib in ${LIBS:-libmano_hip_stamp.so}; do
  echo "== $lib WARM=${WARM:-300}" | tee -a $OUT/log
  timeout -k 10 120 python tools/debug/bs_stamps.py $lib > $OUT/tmp.log 2>&1 || { cat $OUT/tmp.log; exit 1; }
  grep -v amdgpu.ids $OUT/tmp.log | tee -a $OUT/log
done
