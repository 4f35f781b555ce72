#!/bin/bash
# Steady-state check: default bench, then a kernel trace of 400 cold launches
# (no warmup) to see how long the chip takes to reach its steady clock.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/ramp
mkdir -p $OUT
timeout -k 10 300 python bench.py --no-cpu > $OUT/bench.log 2>&1 || { echo "bench rc=$?"; tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o ramp --output-format csv -- python bench.py --steps 400 --warmup 0 --no-cpu > $OUT/prof.log 2>&1 || { echo "prof rc=$?"; tail -5 $OUT/prof.log; exit 1; }
python tools/trace_durations.py $(find $OUT/trace -name '*kernel_trace.csv') blend_skin16 > $OUT/durations.txt
awk 'NR%20==1' $OUT/durations.txt
