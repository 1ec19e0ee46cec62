"""numpy restatement of the HIP kernels' counter-based dropout (k3m_amd/csrc/common.h: k3m_seed_key,
k3m_hash_key, k3m_drop): element ``e`` of a site with (seed, offset) is kept iff
(hash(seed, offset + e) >> 8) >= ceil(p * 2^24), and then scaled by 1 / (1 - p) (fp32).  Attention
probabilities draw one value per key pair (k3m_attn_drop): score (row, j) of a block with lk keys per row takes
the (j & 1) 16-bit half of hash(seed, offset + row * ceil(lk / 2) + j // 2), kept iff >= ceil(p * 2^16).  Test
infrastructure: it regenerates the masks the engine applied so the oracle can be fed the same ones."""
import numpy as np

M64 = (1 << 64) - 1


def seed_key(seed):
    z = (int(seed) + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def hash_ctr(seed, ctr):
    """k3m_hash_key(k3m_seed_key(seed), ctr) for a uint64 array of counters -> uint32 array."""
    key = seed_key(seed)
    ctr = np.asarray(ctr, dtype=np.uint64)
    lo = (ctr & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    hi = (ctr >> np.uint64(32)).astype(np.uint32)
    k_lo, k_hi = np.uint32(key & 0xFFFFFFFF), np.uint32(key >> 32)
    x = lo ^ k_lo ^ ((hi ^ k_hi).astype(np.uint64) * np.uint64(0x9E3779B1) & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    x = x.astype(np.uint64)
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & np.uint64(0xFFFFFFFF)
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & np.uint64(0xFFFFFFFF)
    x ^= x >> np.uint64(16)
    return x.astype(np.uint32)


def keep_scale(seed, off, n, p):
    """float32 [n]: 1/(1-p) where element off+e is kept, 0 where dropped (p == 0: all ones)."""
    if p <= 0:
        return np.ones(n, np.float32)
    thr = np.uint32(np.ceil(np.float32(p) * np.float32(16777216.0)))
    h = hash_ctr(seed, np.uint64(off) + np.arange(n, dtype=np.uint64))
    scale = np.float32(1.0) / (np.float32(1.0) - np.float32(p))
    return np.where((h >> np.uint32(8)) >= thr, scale, np.float32(0.0)).astype(np.float32)


def attn_keep_scale(seed, off, rows, lk, p):
    """float32 [rows * lk] (row-major [row, key]): the attention-probability mask of k3m_attn_drop."""
    if p <= 0:
        return np.ones(rows * lk, np.float32)
    thr = np.uint32(np.ceil(np.float32(p) * np.float32(65536.0)))
    lkp = (lk + 1) // 2
    j = np.arange(lk, dtype=np.uint64)
    ctr = np.uint64(off) + np.arange(rows, dtype=np.uint64)[:, None] * np.uint64(lkp) + (j >> np.uint64(1))[None, :]
    h = hash_ctr(seed, ctr)
    half = np.where((j & np.uint64(1)).astype(bool)[None, :], h >> np.uint32(16), h & np.uint32(0xFFFF))
    scale = np.float32(1.0) / (np.float32(1.0) - np.float32(p))
    return np.where(half >= thr, scale, np.float32(0.0)).astype(np.float32).reshape(-1)
