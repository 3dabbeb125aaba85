"""Host mirror of the reset RNG of the step kernel (csrc/pbg_math.h philox4x32_10).

The reference draws reset noise with gym's np_random (robot_locomotors.py:18-19:
uniform(-0.1, 0.1) per ordered joint).  The batched kernel draws the same distribution
from Philox4x32-10, key = seed, counter = (global env id, episode index, block, 0x5EED),
so that results do not depend on how envs are sharded over GPUs.  This module
reproduces those draws on the host bit-for-bit (trace replay, sharding tests)."""
from __future__ import annotations

import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(ctr, key):
    """ctr: uint32 array [..., 4]; key: (k0, k1).  Returns uint32 [..., 4]."""
    x, y, z, w = [ctr[..., i].astype(np.uint64) for i in range(4)]
    k0, k1 = np.uint64(key[0]), np.uint64(key[1])
    for _ in range(10):
        p0 = M0 * x
        p1 = M1 * z
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK
        x, y, z, w = (hi1 ^ y ^ k0) & MASK, lo1, (hi0 ^ w ^ k1) & MASK, lo0
        k0 = (k0 + np.uint64(W0)) & MASK
        k1 = (k1 + np.uint64(W1)) & MASK
    return np.stack([x, y, z, w], axis=-1).astype(np.uint32)


def reset_noise(seed: int, global_ids, episode, n_reset_dofs: int) -> np.ndarray:
    """float32 [len(global_ids), n_reset_dofs] = the kernel's U(-0.1, 0.1) reset draws."""
    gid = np.asarray(global_ids, dtype=np.uint32)
    epi = np.broadcast_to(np.asarray(episode, dtype=np.uint32), gid.shape)
    key = (seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    out = np.zeros((gid.size, n_reset_dofs), dtype=np.float32)
    for blk in range((n_reset_dofs + 3) // 4):
        ctr = np.stack([gid, epi, np.full_like(gid, blk), np.full_like(gid, 0x5EED)], axis=-1)
        r = philox4x32_10(ctr, key)
        u = (r >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
        # fmaf(0.2f, u, -0.1f): exact in float64, then one rounding to float32
        v = (np.float64(np.float32(0.2)) * u.astype(np.float64) + np.float64(np.float32(-0.1))).astype(np.float32)
        for t in range(4):
            j = 4 * blk + t
            if j < n_reset_dofs:
                out[:, j] = v[:, t]
    return out


def sample_actions(action_dim: int, global_ids, steps, seed: int = 0x5EED) -> np.ndarray:
    """float32 [len(steps), len(global_ids), action_dim] = pbg_sample_actions' U(-1, 1) draws
    (Philox4x32-10, key = seed, counter = (step, global env id, block of 4 actions, 0xAC7))."""
    gid = np.asarray(global_ids, dtype=np.uint32)
    st = np.asarray(steps, dtype=np.uint32)
    key = (seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    out = np.zeros((st.size, gid.size, action_dim), dtype=np.float32)
    S, G = np.meshgrid(st, gid, indexing="ij")
    for blk in range((action_dim + 3) // 4):
        ctr = np.stack([S, G, np.full_like(S, blk), np.full_like(S, 0xAC7)], axis=-1)
        r = philox4x32_10(ctr, key)
        u = (r >> np.uint32(8)).astype(np.float32) * np.float32(1.0 / 16777216.0)
        v = (2.0 * u.astype(np.float64) - 1.0).astype(np.float32)  # fmaf(2, u, -1): exact, one rounding
        for t in range(4):
            j = 4 * blk + t
            if j < action_dim:
                out[..., j] = v[..., t]
    return out
