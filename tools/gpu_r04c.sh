#!/bin/bash
# Round 4 (c): the GPU suite on the product tree, the aligned skin_pair
# (MANO_PAIR_ALIGN=1 build) through the LBS parity tests, then the store-policy
# and aligned-LBS A/B (tools/debug/time_path.py, digests compared there) and the
# default bench.  Every GPU step time-limited; any failure other than a plain
# test failure stops the script, and so does a failing variant suite (its
# timings would be void).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04c}
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/steps.log
  tail -3 "$OUT/$name.log" | cut -c1-600
  if grep -q "HIP error\|illegal memory access\|Memory access fault" "$OUT/$name.log"; then
    echo "stopping: GPU error in $name"; exit 3
  fi
  return $rc
}
PYT="python -u -m pytest -v --timeout 180 --timeout-method thread"
for s in ${STEPS:-tests pairal path bench pmc stats}; do
  case $s in
    tests) step pytest_gpu 900 $PYT tests -m gpu || [ $? -eq 1 ] || exit 1 ;;
    phase) step pytest_phase 300 $PYT tests/test_gpu_parity.py -k "phase_independent or library_is" || exit 1 ;;
    pairal) MANO_TEST_LIB=libmano_hip_pairal.so step pytest_pairal 400 $PYT tests/test_gpu_parity.py \
              -k "standalone_lbs or phase_independent or other_mesh or fused_equals or library_is" || exit 1 ;;
    path) step time_path 900 python tools/debug/time_path.py ${PATH_LIBS:-libmano_hip.so libmano_hip_pairal.so libmano_hip_palnt1.so libmano_hip_palnt2.so libmano_hip_palnt3.so libmano_hip_pnt3.so libmano_hip_restnt1.so libmano_hip_restnt2.so libmano_hip_restnt3.so libmano_hip_bpol0.so libmano_hip_bpol2.so} --reps 2 || exit 1 ;;
    bench) step bench 400 python bench.py --steps 20 --warmup 5 || exit 1 ;;
    pmc)  # blend_skin16 bytes per launch, verts-only and with rest_verts (align_bound.py --loop)
      for lib in ${PMC_LIBS:-libmano_hip.so libmano_hip_legacy.so}; do
        for what in verts rest; do
          for c in WRITE_SIZE FETCH_SIZE; do
            step pmc_${lib%.so}_${what}_$c 90 rocprofv3 --pmc $c -d $OUT/pmc_${lib%.so}_${what}_$c -o p --output-format csv -- python tools/debug/align_bound.py --loop $lib $what 20 || exit 1
          done
        done
      done ;;
    stamps)  # skin_pair per-wave cycle stamps, legacy vs aligned units
      for lib in ${STAMP_LIBS:-libmano_hip_pstamp.so libmano_hip_palstamp.so}; do
        step stamps_${lib%.so} 200 python tools/debug/pair_stamps.py $lib || exit 1
      done ;;
    workloads)  # the other BASELINE configs on one GPU, the 1-rank nccl C4 line, the 2-rank gloo gather rehearsal
      step bench_c5 300 python bench.py --workload C5 --steps 50 --warmup 5 --no-cpu --no-extra || exit 1
      step bench_c3 300 python bench.py --workload C3 --steps 30 --warmup 3 --no-cpu --no-extra || exit 1
      step bench_c4 300 python bench.py --workload C4 --steps 50 --warmup 5 --no-cpu --no-extra || exit 1
      step bench_c4_pg 400 python bench.py --force-pg --workload C4 --steps 20 --warmup 5 --no-extra --no-dropin --cpu-seconds 5 || exit 1
      step bench_c4_dp2 300 python bench.py --gpus 2 --backend gloo --workload C4 --batch 65536 --steps 10 --warmup 3 --no-cpu --no-extra || exit 1 ;;
    probe) step skin_align_probe 400 python tools/debug/skin_align_probe.py --reps 2 || exit 1 ;;
    dist)  # the nccl 1-rank tests (after the ncclFloat change) and 8-rank gloo rehearsals sharing the GPU
      step pytest_dist 400 $PYT tests/test_gpu_distributed.py || exit 1
      step bench_c2_dp8 400 python bench.py --gpus 8 --backend gloo --steps 10 --warmup 3 --no-cpu --no-extra || exit 1
      step bench_c4_dp8 400 python bench.py --gpus 8 --backend gloo --workload C4 --batch 16384 --steps 5 --warmup 2 --no-cpu --no-extra || exit 1 ;;
    clock) step clk 200 env TAG=${TAG:-r04c} LIBS=libmano_hip_stamp.so bash tools/debug/clk_stamps.sh || exit 1 ;;
    fused) step pytest_fused 300 $PYT tests/test_gpu_parity.py -k "fused_equals_unfused" || exit 1 ;;
    dropin) step pytest_dropin 300 $PYT tests/test_gpu_dropin_io.py tests/test_gpu_parity.py -k "dropin or stateful or export_obj" || exit 1
      step dropin_parts 200 python tools/debug/dropin_parts.py || exit 1
      step dropin_latency 200 python tools/debug/dropin_latency.py || exit 1 ;;
    ffi) step pytest_ffi 300 $PYT tests/test_gpu_ffi.py tests/test_abi.py || exit 1
      step ffi_latency 200 python tools/debug/ffi_latency.py || exit 1 ;;
    stats) step kernel_stats 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o k --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu || exit 1 ;;
  esac
done
