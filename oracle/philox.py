"""numpy restatement of the synthetic-workload generator -- TEST INFRASTRUCTURE.

`include/mano_hip.h` (mano_synthetic_inputs) specifies the benchmark's hand
inputs as Philox-4x32-10 (Salmon et al., "Parallel random numbers: as easy as
1, 2, 3", SC'11; the constants below are the published ones) keyed by the
seed, with counter (global hand index lo, hi, block, 0), then Box-Muller.  The
reference has no generator (its demo uses fixed vectors, mano_np.py:209-218);
this module pins the device generator's words bit for bit and its floats to
float32 rounding, so a shard's inputs are provably the global batch's.
"""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(c, k0, k1):
    """c: (..., 4) uint32 counters; k0, k1: uint32 key -> (..., 4) uint32 words."""
    c = [np.asarray(c[..., i], dtype=np.uint32) for i in range(4)]
    k0, k1 = np.uint32(k0), np.uint32(k1)
    with np.errstate(over="ignore"):
        for r in range(10):
            if r > 0:
                k0 = np.uint32(k0 + W0)
                k1 = np.uint32(k1 + W1)
            p0 = M0 * c[0].astype(np.uint64)
            p1 = M1 * c[2].astype(np.uint64)
            hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & MASK).astype(np.uint32)
            hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & MASK).astype(np.uint32)
            c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
    return np.stack(c, axis=-1)


def words(seed, first, n):
    """The 64 uint32 words of hands first..first+n-1: (n, 64)."""
    g = np.arange(first, first + n, dtype=np.uint64)
    ctr = np.zeros((n, 16, 4), dtype=np.uint32)
    ctr[..., 0] = (g & MASK).astype(np.uint32)[:, None]
    ctr[..., 1] = (g >> np.uint64(32)).astype(np.uint32)[:, None]
    ctr[..., 2] = np.arange(16, dtype=np.uint32)[None, :]
    return philox4x32_10(ctr, np.uint64(seed) & MASK, np.uint64(seed) >> np.uint64(32)).reshape(n, 64)


def unit_open(w):
    """((w >> 8) + 0.5) / 2^24, in (0, 1)."""
    return ((w >> np.uint32(8)).astype(np.float64) + 0.5) / 16777216.0


def synthetic_inputs(seed, first, n, beta_sigma=1.0, pose_sigma=0.5, trans_range=1.0):
    """float64 values of mano_synthetic_inputs: betas (n,10), pose (n,16,3), trans (n,3)."""
    w = words(seed, first, n)
    u = unit_open(w)
    r = np.sqrt(-2.0 * np.log(u[:, 0:58:2]))
    phi = 2.0 * np.pi * u[:, 1:58:2]
    normals = np.empty((n, 58))
    normals[:, 0::2] = r * np.cos(phi)
    normals[:, 1::2] = r * np.sin(phi)
    return {"betas": beta_sigma * normals[:, :10],
            "pose": pose_sigma * normals[:, 10:58].reshape(n, 16, 3),
            "trans": trans_range * (2.0 * u[:, 58:61] - 1.0)}
