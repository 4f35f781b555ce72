set -u
mkdir -p gpurun_out/ring
timeout -k 10 120 python tools/debug/time_skin.py > gpurun_out/ring/time_ring.log 2>&1; rc=$?; cat gpurun_out/ring/time_ring.log | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_f16x3.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ring/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/ring/pytest.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 120 python tools/debug/time_skin.py libmano_hip_span.so 2>&1 | grep -v amdgpu.ids
timeout -k 10 120 python tools/debug/time_skin.py 2>&1 | grep -v amdgpu.ids
