#!/bin/bash
# Time stage_skin for each library build given (debug builds in mano_amd/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/variants
for lib in "$@"; do
  timeout -k 10 180 python -u tools/debug/${TIMER:-time_skin}.py $lib >> gpurun_out/variants/skin.log 2>&1 || { rc=$?; tail -5 gpurun_out/variants/skin.log; exit $rc; }
done
grep -v amdgpu.ids gpurun_out/variants/skin.log
