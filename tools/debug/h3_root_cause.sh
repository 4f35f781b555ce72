#!/bin/bash
# Root cause of the round-1 f16x3 fault: build the failing
# configuration (SLP on, no_pack transparent) and the same with every counted
# vmcnt barrier replaced by vmcnt(0), here on the CPU:
#   bash tools/debug/h3_root_cause.sh build
# then on the GPU box:
#   bash tools/debug/h3_root_cause.sh run
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
PKG=mano-hand_amd
SRCS="$PKG/csrc/mano_abi.hip $PKG/csrc/mano_comm.hip $PKG/csrc/mano_pack.cpp $PKG/csrc/mano_articulate.hip $PKG/csrc/mano_kernels.hip $PKG/csrc/mano_kernels_h3.hip $PKG/csrc/mano_skin_quad.hip"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ldl -DMANO_DIAGNOSTIC_BUILD=1"
if [ "${1:-}" = build ]; then
  /opt/rocm/bin/hipcc $FLAGS -DMANO_H3_NO_PACK=0 -o $PKG/mano_amd/libmano_hip_pack.so $SRCS
  /opt/rocm/bin/hipcc $FLAGS -DMANO_H3_NO_PACK=0 -DMANO_H3_FULL_WAIT=1 -o $PKG/mano_amd/libmano_hip_pack_fullwait.so $SRCS
  # every instruction preceded by s_nop 7: no instruction-level hazard can survive
  /opt/rocm/bin/hipcc $FLAGS -DMANO_H3_NO_PACK=0 -mllvm -amdgpu-snop-padding=7 -o $PKG/mano_amd/libmano_hip_pack_snop.so $SRCS
  # every wait the compiler emits is a full wait, and the hand-counted barriers too: no memory-timing race
  /opt/rocm/bin/hipcc $FLAGS -DMANO_H3_NO_PACK=0 -DMANO_H3_FULL_WAIT=1 -mllvm -amdgpu-waitcnt-forcezero -o $PKG/mano_amd/libmano_hip_pack_zero.so $SRCS
  # packed everywhere except the final fma(o, 2^-k, trans) of the LBS output
  /opt/rocm/bin/hipcc $FLAGS -DMANO_H3_NO_PACK=0 -DMANO_H3_SCALAR_UNSCALE=1 -o $PKG/mano_amd/libmano_hip_pack_su.so $SRCS
  ls -la $PKG/mano_amd/libmano_hip_pack*.so
else
  OUT=gpurun_out/${TAG:-h3rc}
  mkdir -p $OUT
  [ -n "${MFMA_RAW:-}" ] && timeout -k 10 120 ./tools/microbench/mfma_raw > $OUT/mfma_raw.log 2>&1
  for lib in ${LIBS:-libmano_hip_pack.so libmano_hip_pack_fullwait.so libmano_hip_pack_snop.so libmano_hip_pack_zero.so libmano_hip.so}; do
    timeout -k 10 120 python tools/debug/h3_fused_variants.py $lib > $OUT/variants_$lib.log 2>&1
    echo "== $lib"; cat $OUT/variants_$lib.log
  done
fi
