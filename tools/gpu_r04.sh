#!/bin/bash
# Round 4 GPU session: the GPU suite, the aligned-store bound (align_bound.py
# A/B + WRITE_SIZE / FETCH_SIZE passes), the default bench and the 1-rank
# RCCL C4 line.  Every GPU step time-limited; stop on a fault / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  tail -3 "$OUT/$name.log" | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  return 0
}
for s in ${STEPS:-tests align pmc bench c4}; do
  case $s in
    tests) step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread ${PYTEST_ARGS:-} ;;
    align) step align_bound 500 python tools/debug/align_bound.py ${ALIGN_LIBS:-libmano_hip.so libmano_hip_abl4.so} --reps 3 ;;
    pmc)
      for lib in ${PMC_LIBS:-libmano_hip.so libmano_hip_abl4.so}; do
        for what in verts rest; do
          for c in WRITE_SIZE FETCH_SIZE; do
            step pmc_${lib%.so}_${what}_$c 90 rocprofv3 --pmc $c -d $OUT/pmc_${lib%.so}_${what}_$c -o p --output-format csv -- python tools/debug/align_bound.py --loop $lib $what 20
          done
        done
      done ;;
    path) step time_path 600 python tools/debug/time_path.py ${PATH_LIBS:-libmano_hip.so} --reps 2 ;;
    pmcblend)
      for lib in ${PMC_LIBS:-libmano_hip.so}; do
        for c in WRITE_SIZE FETCH_SIZE; do
          MANO_LIB=$lib step pmcu_${lib%.so}_$c 90 rocprofv3 --pmc $c -d $OUT/pmcu_${lib%.so}_$c -o p --output-format csv -- python tools/debug/run_path.py unfused 20
        done
      done ;;
    probe) step skin_align_probe 400 python tools/debug/skin_align_probe.py --reps 2 ;;
    bench) step bench 400 python bench.py --steps 20 --warmup 5 ;;
    c4) step bench_c4_pg 400 python bench.py --force-pg --workload C4 --steps 20 --warmup 5 --no-extra --no-dropin --cpu-seconds 5 ;;
    *) if [ -n "${EXTRA:-}" ]; then step extra 400 bash -c "$EXTRA"; fi ;;
  esac
done
