TAG=r03_pmc bash tools/pmc_path.sh unfused skin_b2b staged rest_verts > gpurun_out/r03_pmc.log 2>&1 || { tail -20 gpurun_out/r03_pmc.log; exit 1; }
tail -12 gpurun_out/r03_pmc.log
mkdir -p gpurun_out/r03d
timeout -k 10 600 python tools/debug/time_path.py libmano_hip.so libmano_hip_sst.so libmano_hip_sst2.so --reps 2 > gpurun_out/r03d/ab_sst.log 2>&1; rc=$?
cut -c1-400 gpurun_out/r03d/ab_sst.log
exit $rc
