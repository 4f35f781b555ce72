set -u
mkdir -p gpurun_out/acc2
for rep in 1 2 3; do
  for lib in libmano_hip.so libmano_hip_acc2.so; do
    timeout -k 10 120 python tools/debug/time_stages.py $lib 2>&1 | grep -v amdgpu.ids >> gpurun_out/acc2/times.log || exit 1
  done
done
