#!/bin/bash
# blend_skin16 ablations (diagnostic): build here with `build`, time on the GPU box with `run`.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
PKG=mano-hand_amd
SRCS="$PKG/csrc/mano_abi.hip $PKG/csrc/mano_comm.hip $PKG/csrc/mano_pack.cpp $PKG/csrc/mano_articulate.hip $PKG/csrc/mano_kernels.hip $PKG/csrc/mano_kernels_h3.hip $PKG/csrc/mano_skin_quad.hip"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ldl -fno-slp-vectorize"
VARIANTS=${VARIANTS:-"abl1:-DMANO_BS_ABLATE=1 abl2:-DMANO_BS_ABLATE=2 abl3:-DMANO_BS_ABLATE=3"}
if [ "${1:-}" = build ]; then
  for v in $VARIANTS; do
    name=${v%%:*}; defs=${v#*:}
    python -c "import sys, __graft_entry__ as g; g.build_library('$PKG/mano_amd/libmano_hip_$name.so', sys.argv[1:])" ${defs//,/ } &
  done
  wait
  ls -la $PKG/mano_amd/libmano_hip_*.so
else
  OUT=gpurun_out/${TAG:-ablate}; mkdir -p $OUT
  for rep in 1 2; do
    for lib in libmano_hip.so $(for v in $VARIANTS; do echo libmano_hip_${v%%:*}.so; done); do
      VERTS_ROW=1072 timeout -k 10 120 python tools/debug/time_forward.py $lib 2>&1 | grep -v amdgpu.ids | tee -a $OUT/times.log
    done
  done
fi
