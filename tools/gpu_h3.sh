#!/bin/bash
# f16x3 iteration: its GPU tests, then both benches (no CPU baseline).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/h3
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_f16x3.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -15 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu --precision f16x3 > $OUT/bench_h3.log 2>&1 || { rc=$?; tail -5 $OUT/bench_h3.log; exit $rc; }
tail -1 $OUT/bench_h3.log
timeout -k 10 300 python bench.py --no-cpu > $OUT/bench_fp32.log 2>&1 || { rc=$?; tail -5 $OUT/bench_fp32.log; exit $rc; }
tail -1 $OUT/bench_fp32.log
