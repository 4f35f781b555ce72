#!/bin/bash
# Round 6 GPU steps, each time-limited; stop on the first fault / timeout.
#   STEPS="tests bench dp8" TAG=r06a bash tools/gpu_r06.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/steps.log
  local t0=$(date +%s%N)
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  local t1=$(date +%s%N)
  echo "=== $name rc=$rc wall_ms=$(( (t1 - t0) / 1000000 ))" | tee -a $OUT/steps.log
  tail -3 "$OUT/$name.log" | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
  if [ $rc -eq 1 ] && [ "${STOP_ON_FAIL:-1}" = 1 ]; then echo "stopping after rc=1"; exit 1; fi
  return 0
}
for s in ${STEPS:-tests bench}; do
  case $s in
    tests) step pytest_gpu 1100 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread ${PYTEST_ARGS:-} ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 500 python bench.py --steps 20 --warmup 5 ;;
    # the driver's N = 8 command, rehearsed with 8 gloo ranks sharing this
    # box's one GPU, every rank-0 leg on (the CPU baseline at the box's
    # 16-core share instead of cpu_share(8) = 128)
    dp8) step bench_dp8 600 python bench.py --gpus 8 --backend gloo --steps 20 --warmup 5 --cpu-procs 16 ;;
    # round 6: the in-place LBS (parity, then the A/B against the separate form)
    inplace_tests) step pytest_inplace 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_codegen.py -m gpu -x -v --timeout 180 --timeout-method thread -k "in_place or standalone or fused_equals or codegen or isa" ;;
    inplace_ab) step inplace_ab 400 python tools/debug/time_inplace.py libmano_hip.so libmano_hip_ipfwd.so --reps 2 ;;
    inplace_span) step inplace_span 400 python tools/debug/time_inplace.py libmano_hip.so libmano_hip_ipspan.so --reps 3 ;;
    inplace_hot) step inplace_hot 500 python tools/debug/time_inplace.py libmano_hip.so libmano_hip_iphot.so --reps 3 ;;
    inplace_hot2) step inplace_hot2 600 python tools/debug/time_inplace.py libmano_hip.so libmano_hip_iphot.so libmano_hip_iphots.so libmano_hip_iphotr.so --reps 2 ;;
    inplace_final) step inplace_final 500 python tools/debug/time_inplace.py libmano_hip.so libmano_hip_iphot0.so --reps 3 ;;
    inplace_nt) step inplace_nt 500 python tools/debug/time_inplace.py libmano_hip.so libmano_hip_ipnt1.so libmano_hip_ipnt2.so libmano_hip_ipnt3.so --reps 2 ;;
    # the driver's N = 8 command with the multi-GPU legs (C3 2^24 and C4 2^22
    # at their BASELINE sizes), 8 gloo ranks sharing this box's GPU
    dp8legs) step bench_dp8_legs 600 python bench.py --gpus 8 --backend gloo --steps 20 --warmup 5 --cpu-procs 16 ;;
    # the RCCL form of the multi-GPU legs at BASELINE sizes, one rank (C3: the
    # whole 2^24 batch on this GPU; C4: 2^22 + mano_gather + the ring copy)
    legs1) step bench_legs1 600 python bench.py --force-pg --backend nccl --legs on --steps 20 --warmup 5 --no-cpu --no-dropin ;;
    dist_tests) step pytest_dist 600 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_multi_device.py -m gpu -x -v --timeout 180 --timeout-method thread ;;
    pg1) step bench_pg1 300 python bench.py --force-pg --backend nccl --steps 20 --warmup 5 --no-cpu --no-dropin --legs off ;;
    # kernel traces of the timed steps: N = 1, and one rank under a process group (nccl, gloo)
    trace_pg) B="python bench.py --steps 20 --warmup 5 --no-extra --no-check --no-dropin --no-cpu --no-live-pmc"
       step trace_n1 300 rocprofv3 --kernel-trace -d $OUT/tr_n1 -o t --output-format csv -- $B
       WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29611 step trace_nccl 300 rocprofv3 --kernel-trace -d $OUT/tr_nccl -o t --output-format csv -- $B --force-pg --backend nccl --legs off
       WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29612 step trace_gloo 300 rocprofv3 --kernel-trace -d $OUT/tr_gloo -o t --output-format csv -- $B --force-pg --backend gloo --legs off
       for t in n1 nccl gloo; do echo "$t $(python tools/trace_steps.py $OUT/tr_$t)"; done | tee $OUT/trace_steps.txt ;;
    # the process group's cost on one GPU: plain, gloo group, nccl group alternating
    pg_ab) F="--steps 20 --warmup 5 --no-extra --no-check --no-dropin --no-cpu --no-live-pmc --legs off"
       for i in 1 2 3; do
         step ab_plain_$i 120 python bench.py $F
         step ab_gloo_$i 120 python bench.py $F --force-pg --backend gloo
         step ab_nccl_$i 120 python bench.py $F --force-pg --backend nccl
       done
       for f in $OUT/ab_*.log; do echo "$(basename $f) $(grep '^{' $f | tail -1 | python -c 'import json,sys; l=json.load(sys.stdin); k=l["kernels"]; print(round(l["ms_per_step"],4), round(k["articulate"]["ms"],4), round(k["blend_skin"]["ms"],4))')"; done | tee $OUT/pg_ab.txt ;;
    stats) step stats 500 rocprofv3 --kernel-trace --stats -d $OUT/stats -o bench --output-format csv -- python bench.py --no-cpu ;;
    *) step extra_$s 600 bash -c "$s" ;;
  esac
done
