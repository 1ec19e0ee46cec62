"""The numpy restatement of the kernels' dropout draws (tests/dropmask.py, k3m_amd/csrc/common.h), on the CPU: the
attention-probability mask draws one 32-bit value per key pair (k3m_attn_drop), the hidden-state mask one per element
(k3m_drop).  The GPU side is pinned against these by tests/test_gpu_train_mode_parity.py."""
import numpy as np

import dropmask as DM


def _attn_ref(seed, off, rows, lk, p):
    """k3m_attn_drop element by element: (row, j) takes the (j & 1) half of hash(off + row * ceil(lk / 2) + j // 2)."""
    thr = int(np.ceil(np.float32(p) * np.float32(65536.0)))
    scale = np.float32(1.0) / (np.float32(1.0) - np.float32(p))
    out = np.zeros((rows, lk), np.float32)
    lkp = (lk + 1) // 2
    for r in range(rows):
        for j in range(lk):
            h = int(DM.hash_ctr(seed, np.array([off + r * lkp + j // 2], np.uint64))[0])
            half = (h >> 16) if (j & 1) else (h & 0xFFFF)
            out[r, j] = scale if half >= thr else 0.0
    return out.reshape(-1)


def test_attn_mask_matches_elementwise_definition():
    for lk in (1, 7, 36, 37):   # odd key counts: the last pair has one live key
        got = DM.attn_keep_scale(1234, 99, 5, lk, 0.1)
        assert np.array_equal(got, _attn_ref(1234, 99, 5, lk, 0.1)), lk


def test_attn_mask_pairs_share_one_draw_and_rows_do_not():
    seed, off, rows, lk = 7, 1 << 33, 64, 320   # an offset past 2^32: the counter's high word is used
    m = DM.attn_keep_scale(seed, off, rows, lk, 0.1).reshape(rows, lk)
    lkp = (lk + 1) // 2
    ctr = np.uint64(off) + np.arange(rows, dtype=np.uint64)[:, None] * np.uint64(lkp) + \
        (np.arange(lk, dtype=np.uint64) >> np.uint64(1))[None, :]
    h = DM.hash_ctr(seed, ctr)
    assert np.array_equal(h[:, 0::2], h[:, 1::2])   # keys 2m and 2m + 1 read the same 32-bit draw
    assert not np.array_equal(m[0], m[1])


def test_attn_mask_rate_and_scale():
    p = 0.1
    m = DM.attn_keep_scale(42, 0, 2048, 320, p)
    kept = m != 0
    assert abs(kept.mean() - (1 - p)) < 3e-3        # 655,360 draws: 5 sigma ~ 1.9e-3
    assert np.allclose(m[kept], 1 / (1 - np.float32(p)))
    assert np.array_equal(DM.attn_keep_scale(42, 0, 3, 5, 0.0), np.ones(15, np.float32))


def test_hidden_mask_is_per_element():
    p = 0.1
    m = DM.keep_scale(5, 77, 200000, p)
    assert abs((m != 0).mean() - (1 - p)) < 4e-3
    # neighbouring elements keep independently: agreement (1 - p)^2 + p^2
    agree = np.mean((m[0::2] != 0) == (m[1::2] != 0))
    assert abs(agree - ((1 - p) ** 2 + p ** 2)) < 6e-3
