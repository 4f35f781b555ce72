#!/bin/bash
# Round-end evidence: smoke, the default bench (with CPU baseline), and the
# rocprofv3 kernel-trace stats of the same default bench command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/final
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { rc=$?; tail -5 $OUT/smoke.log; exit $rc; }
echo smoke ok
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || { rc=$?; tail -5 $OUT/bench.log; exit $rc; }
tail -1 $OUT/bench.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/stats -o bench --output-format csv -- python bench.py --no-cpu > $OUT/stats.log 2>&1 || { rc=$?; tail -5 $OUT/stats.log; exit $rc; }
echo stats ok
