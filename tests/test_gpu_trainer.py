"""The optimizer and sampler kernels and the Trainer's A14 features on the GPU:

* k3m_adamw_ex (pytorch_transformers AdamW / apex FusedAdam, fused zero_grad) against the oracle's
  restatements, element for element;
* k3m_lpm_sample: draws without replacement, k != i, j' != j, counts min(#candidates, n) for any
  num_negative_pv (vilbert_k3m.py:2476-2492), roughly uniform;
* num_negative_pv = 10 through the whole forward, checked against the oracle fed the same draws;
* gradient accumulation (train_concap_struc.py:561-575): the first moment after two micro-steps is
  (1 - beta1) times the mean of the two micro-batch gradients;
* NaN fail-fast on a batch with no masked region (the reference's 0/0 region loss).
"""
import math

import numpy as np
import pytest
import torch

from golden_util import CFG_PATH, load_case, case_config, case_batch, case_noise

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda")


@pytest.mark.parametrize("flags", [0, 1, 2, 3, 6])
def test_adamw_ex_matches_restatement(dev, flags):
    from k3m_amd import _lib as L
    from oracle.k3m_oracle import adamw_step, fused_adam_step
    n = 4096 + 128
    gen = torch.Generator().manual_seed(flags)
    p = torch.randn(n, generator=gen)
    g = torch.randn(n, generator=gen) * 0.1
    m = torch.randn(n, generator=gen) * 0.01
    v = torch.rand(n, generator=gen) * 1e-3
    pd, gd, md, vd = p.to(dev), g.to(dev), m.to(dev), v.to(dev)
    sh = torch.empty(n, dtype=torch.bfloat16, device=dev)
    step, lr, wd, b1, b2 = 3, 1e-3, 0.01, 0.9, (0.999 if flags & 2 else 0.98)
    L.call("k3m_adamw_ex", pd.data_ptr(), gd.data_ptr(), md.data_ptr(), vd.data_ptr(), sh.data_ptr(), n, lr, b1, b2,
           1e-8, wd, step, 0.5, flags, L.stream())
    torch.cuda.synchronize()
    gs = g * 0.5
    if flags & 2:
        fused_adam_step(p, gs, m, v, step, lr, wd, beta1=b1, beta2=b2, eps=1e-8, bias_correction=bool(flags & 4))
    else:
        adamw_step(p, gs, m, v, step, lr, wd, beta1=b1, beta2=b2, eps=1e-8)
    np.testing.assert_allclose(pd.cpu().numpy(), p.numpy(), rtol=2e-6, atol=1e-7)
    np.testing.assert_allclose(md.cpu().numpy(), m.numpy(), rtol=2e-6, atol=1e-9)
    np.testing.assert_allclose(vd.cpu().numpy(), v.numpy(), rtol=2e-6, atol=1e-12)
    assert torch.equal(sh.cpu(), pd.cpu().to(torch.bfloat16))
    if flags & 1:
        assert float(gd.abs().max()) == 0.0
    else:
        assert torch.equal(gd.cpu(), g)


@pytest.mark.parametrize("ke,kv", [(2, 2), (5, 5), (1, 0), (0, 3), (8, 8)])
def test_lpm_sample_properties(dev, ke, kv):
    from k3m_amd import _lib as L
    B, NPV = 24, 20
    gen = torch.Generator().manual_seed(ke * 10 + kv)
    nvalid = torch.randint(0, NPV + 1, (B,), generator=gen, dtype=torch.int32)
    nvalid[0], nvalid[1] = 0, 1
    nv = nvalid.to(dev)
    ent = torch.empty((B, NPV, ke), dtype=torch.int64, device=dev)
    val = torch.empty((B, NPV, kv), dtype=torch.int64, device=dev)
    counts = np.zeros((B, B), np.int64)
    for s in range(40):
        L.call("k3m_lpm_sample", nv.data_ptr(), B, NPV, ke, kv, 1000 + s, s * 7919, L.ptr(ent), L.ptr(val), L.stream())
        torch.cuda.synchronize()
        E, V = ent.cpu().numpy(), val.cpu().numpy()
        for i in range(B):
            n = int(nvalid[i])
            for j in range(NPV):
                e, v = E[i, j], V[i, j]
                if j >= n:
                    assert (e == -1).all() and (v == -1).all()
                    continue
                te, tv = min(B - 1, ke), min(n - 1, kv)
                assert (e[te:] == -1).all() and (v[tv:] == -1).all()
                de, dv = e[:te], v[:tv]
                assert len(set(de.tolist())) == te and len(set(dv.tolist())) == tv      # without replacement
                assert ((de >= 0) & (de < B) & (de != i)).all()                          # k != i
                assert ((dv >= 0) & (dv < n) & (dv != j)).all()                          # j' != j
                for k in de:
                    counts[i, k] += 1
    if ke:
        # every other item is drawn about equally often (uniform without replacement)
        for i in range(B):
            if int(nvalid[i]) < 10:
                continue
            c = np.delete(counts[i], i).astype(np.float64)
            mu = c.mean()    # binomial spread: every count within 5 standard deviations of the mean
            assert (np.abs(c - mu) <= 5.0 * np.sqrt(mu) + 1.0).all(), (i, c)


def test_num_negative_pv_10_matches_oracle(dev):
    """num_negative_pv = 10 (5 entity + 5 value negatives per triple), drawn on the device, then the
    oracle restatement fed the same draws: losses agree to 1e-3."""
    from k3m_amd.engine import K3MEngine
    from k3m_amd.weights import param_values
    from oracle import k3m_oracle as O
    g = load_case("bs3_zero_triple")
    cfg = case_config(g)
    cfg.num_negative_pv = 10
    eng = K3MEngine(cfg, dev)
    vals = param_values(cfg, int(g["weight_seed"]))
    eng.fp.load(vals)
    batch = case_batch(g)
    noise = case_noise(g)
    out, ctx = eng.forward({k: v.to(dev) for k, v in batch.items()}, train=False,
                           noise={k: v.to(dev) for k, v in noise.items()})
    ent, val = ctx["struct"][8].cpu(), ctx["struct"][9].cpu()
    assert ent.shape[2] == 5 and val.shape[2] == 5
    # 3 items: at most 2 entity candidates each; every valid triple of an item with n triples gets min(n-1, 5)
    assert int((ent[:, :, 2:] >= 0).sum()) == 0 and int((ent[:, :, :2] >= 0).sum()) > 0
    nvalid = ctx["struct"][1].cpu()
    for i in range(3):
        n = int(nvalid[i])
        assert ((val[i, :n] >= 0).sum(-1) == min(max(n - 1, 0), 5)).all()
    P = {k: torch.from_numpy(v) for k, v in vals.items()}
    torch.set_num_threads(16)
    with torch.no_grad():
        ref = O.forward(P, cfg, batch, noise, ent, val)
    for k in ("loss_lpm", "masked_lm_loss", "masked_img_loss", "masked_lm_loss_pv", "loss"):
        a, b = float(out[k]), float(ref[k])
        assert abs(a - b) <= 1e-3 * max(1.0, abs(b)), (k, a, b)


def _no_dropout_cfg():
    from k3m_amd.config import pretrain_config
    cfg = pretrain_config(CFG_PATH)
    cfg.hidden_dropout_prob = cfg.attention_probs_dropout_prob = 0.0
    cfg.v_hidden_dropout_prob = cfg.v_attention_probs_dropout_prob = 0.0
    return cfg


def _fixed_negs(B, NPV, nt):
    ent = torch.full((B, NPV, 2), -1, dtype=torch.int64)
    val = torch.full((B, NPV, 2), -1, dtype=torch.int64)
    for i in range(B):
        for j in range(nt):
            ent[i, j, 0] = (i + 1) % B
            val[i, j, 0], val[i, j, 1] = (j + 1) % nt, (j + 2) % nt
    return ent, val


def test_gradient_accumulation(dev):
    from k3m_amd.trainer import Trainer
    from k3m_amd.synthetic import synthetic_batch, synthetic_noise
    cfg = _no_dropout_cfg()
    B = 3
    batches = [synthetic_batch(cfg, B, dev, seed=s) for s in (21, 22)]
    noises = [{k: v.to(dev) for k, v in synthetic_noise(cfg, B, seed=s).items()} for s in (31, 32)]
    ent, val = _fixed_negs(B, 20, 10)
    ref = Trainer(cfg, dev, lr=1e-3, warmup_steps=0, total_steps=10, seed=5, nan_check=False)
    eng = ref.engine
    acc = torch.zeros_like(eng.fp.grad)
    for b, nz in zip(batches, noises):
        eng.fp.grad.zero_()
        out, ctx = eng.forward(b, train=True, noise=nz, ent_neg=ent, val_neg=val)
        eng.backward(ctx)
        acc += eng.fp.grad
    acc *= 0.5
    want = acc[:ref.m.numel()].clone()
    del ref, eng
    tr = Trainer(cfg, dev, lr=1e-3, warmup_steps=0, total_steps=10, seed=5, accum_steps=2)
    p0 = tr.engine.fp.data.clone()
    tr.step(batches[0], noise=noises[0], ent_neg=ent, val_neg=val)
    assert tr.global_step == 0 and torch.equal(tr.engine.fp.data, p0)        # no update after micro-step 1
    tr.step(batches[1], noise=noises[1], ent_neg=ent, val_neg=val)
    assert tr.global_step == 1
    mask = torch.zeros_like(want, dtype=torch.bool)
    for a, n, _, _ in tr.runs:
        mask[a:a + n] = True
    got = tr.m[mask] / 0.1
    exp = want[mask]
    err = float((got - exp).abs().max())
    assert err <= 1e-5 * float(exp.abs().max()) + 1e-9, err
    assert float(tr.engine.fp.grad.abs().max()) == 0.0      # zero_grad fused into the optimizer sweep
    tr.watch.flush()


def test_nan_loss_fails_fast(dev):
    """No masked region in the batch: the reference's region loss is 0/0 = NaN (:2758-2760); the
    trainer raises instead of updating the model with NaN gradients for ever."""
    from k3m_amd.trainer import Trainer
    from k3m_amd.synthetic import synthetic_batch
    cfg = _no_dropout_cfg()
    tr = Trainer(cfg, dev, lr=1e-4, warmup_steps=0, total_steps=10, seed=5)
    b = synthetic_batch(cfg, 2, dev, seed=3)
    b["image_label"] = torch.full_like(b["image_label"], -1)
    with pytest.raises(FloatingPointError):
        tr.step(b)
        tr.watch.flush()


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_overlapped_optimizer_bit_identical(dev, dtype, deterministic):
    """The per-block AdamW on the side stream (Trainer.overlap, K3M_OPT_OVERLAP) updates every element exactly as
    the one sweep after the backward (AdamW is elementwise; the blocks only re-cut the runs).  Two checks:
    * mechanics, bit-exact: the gradients each block's AdamW consumed are captured at hand-off; a twin trainer
      restored to the same pre-step state runs the one sweep on exactly those gradients, and parameters, both
      moments and the bf16 shadow agree bit for bit after each of three steps; every optimised element is
      covered by exactly one block run; the gradient buffer is zero afterwards;
    * hand-off timing, bit-exact: under K3M_DETERMINISTIC (the fixed-order embedding / structure-aggregator / LPM
      backward) the captured gradients equal a sweep run's final gradients, i.e. no block was read before the
      backward finished it.  (With the float-atomic backward this compared to a tolerance, 1e-3 of each tensor's
      max + 1e-8, which the structure head's output bias -- a gradient that is zero up to rounding, its scores
      entering a softmax -- exceeded once by run-to-run rounding alone: 1.24e-8.)"""
    from k3m_amd.trainer import Trainer
    from k3m_amd.synthetic import synthetic_batch, synthetic_noise
    cfg = _no_dropout_cfg()
    B = 2
    batches = [synthetic_batch(cfg, B, dev, seed=s) for s in (41, 42, 43)]
    noises = [{k: v.to(dev) for k, v in synthetic_noise(cfg, B, seed=s).items()} for s in (51, 52, 53)]
    ent, val = _fixed_negs(B, 20, 10)

    def mk(overlap):
        tr = Trainer(cfg, dev, lr=1e-3, warmup_steps=1, total_steps=10, seed=5, dtype=dtype, nan_check=False)
        tr.overlap = overlap
        return tr

    ta, tb, tc = mk(True), mk(False), mk(False)
    fa, fb, fc = ta.engine.fp, tb.engine.fp, tc.engine.fp
    cap = torch.zeros_like(fa.grad)
    orig = ta._overlap_block

    def capture(blk):
        if blk in ta._pending:
            for a, n, _, _ in ta.block_runs[blk]:
                cap[a:a + n].copy_(fa.grad[a:a + n])   # before orig() records the hand-off event
        orig(blk)
    ta._overlap_block = capture
    final_c = []
    orig_c = tc.optimizer_step

    def grab(*a, **k):
        final_c.append(fc.grad.clone())
        return orig_c(*a, **k)
    tc.optimizer_step = grab
    for k, (b, nz) in enumerate(zip(batches, noises)):
        pre = (fa.data.clone(), ta.m.clone(), ta.v.clone(), fa.data16.clone() if fa.data16 is not None else None)
        ta.step(b, noise=nz, ent_neg=ent, val_neg=val)
        tc.step(b, noise=nz, ent_neg=ent, val_neg=val)
        fb.data.copy_(pre[0])
        tb.m.copy_(pre[1])
        tb.v.copy_(pre[2])
        if pre[3] is not None:
            fb.data16.copy_(pre[3])
        fb.shadow_fresh = fa.shadow_fresh
        tb.global_step = k
        fb.grad.copy_(cap)
        tb.optimizer_step()
        torch.cuda.synchronize()
        assert ta.global_step == k + 1 and float(fa.grad.abs().max()) == 0.0
        assert torch.equal(fa.data, fb.data), k
        assert torch.equal(ta.m, tb.m) and torch.equal(ta.v, tb.v), k
        if fa.data16 is not None:   # over the optimised runs (the forward refreshes the rest of the shadow)
            for a, n, _, _ in ta.runs:
                assert torch.equal(fa.data16[a:a + n], fb.data16[a:a + n]), (k, a, n)
        bad = []
        for name, shape in fa.spec:
            o = fa.offsets[name]
            n = math.prod(shape)
            x, y = cap[o:o + n], final_c[k][o:o + n]
            if not torch.equal(x, y):
                bad.append((name, float((x - y).abs().max()), float(y.abs().max())))
        assert not bad, (k, bad[:10])
    cover = torch.zeros(fa.data.numel(), dtype=torch.int32)
    for runs in ta.block_runs.values():
        for a, n, _, _ in runs:
            cover[a:a + n] += 1
    whole = torch.zeros_like(cover)
    for a, n, _, _ in ta.runs:
        whole[a:a + n] = 1
    assert int(cover.max()) == 1 and torch.equal(cover.bool(), whole.bool())


@pytest.fixture
def deterministic():
    from k3m_amd import ops
    old = ops.DETERMINISTIC
    ops.set_deterministic(True)
    yield
    ops.set_deterministic(old)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_deterministic_step_bit_identical(dev, dtype, deterministic, layout="default"):
    """K3M_DETERMINISTIC: with the fixed-order embedding / structure-aggregator / LPM backward the whole
    training step is bit-reproducible -- two trainers from the same state (dropout, device gumbel noise and
    device-drawn LPM negatives on) end bit-identical after three steps: parameters, both moments, the bf16 shadow.
    And the overlapped per-block AdamW (Trainer.overlap) equals the one sweep after the backward bit for bit over
    the whole step, in both dtypes.  layout (test_deterministic_overlap_layouts): the config-5
    shapes (PV 320 on the long-attention kernels, 50 triples) and the reference's pretrained-model parameter groups
    (per-tensor lr multipliers, frozen embeddings and first text layers: train_concap_struc.py:255-257, :352-389),
    where a block released to the side-stream AdamW before its backward finished would show."""
    from k3m_amd.trainer import Trainer
    from k3m_amd.synthetic import synthetic_batch
    from k3m_amd.config import pretrain_config
    from k3m_amd.engine import label_counts
    cfg = pretrain_config(CFG_PATH)
    B = 4 if layout != "cfg5" else 2
    shape = dict(n_triples=6) if layout != "cfg5" else dict(P=320, n_triples=50, npv=50)
    batches = []
    for s in (61, 62, 63):
        b = synthetic_batch(cfg, B, dev, seed=s, **shape)
        b["_label_counts"] = label_counts(b)
        batches.append(b)
    kw = {}
    if layout == "groups":
        from k3m_amd.params import flat_layout
        names = [n for n, _ in flat_layout(cfg)[0]]
        kw["frozen_names"] = tuple(n for n in names if n.startswith("embeddings.") or n.startswith("encoder.layer.0."))
        kw["lr_mult"] = {n: 0.1 for n in names if n.startswith("encoder.layer.") and n not in kw["frozen_names"]}

    def run(overlap):
        tr = Trainer(cfg, dev, lr=1e-3, warmup_steps=1, total_steps=10, seed=11, dtype=dtype, **kw)
        tr.overlap = overlap
        tr.graph = False
        assert tr.dropout
        for b in batches:
            tr.step(b)
        torch.cuda.synchronize()
        fp = tr.engine.fp
        return (fp.data.clone(), tr.m.clone(), tr.v.clone(), fp.data16.clone() if fp.data16 is not None else None)
    a1, a2, s1 = run(True), run(True), run(False)
    for x, y, z in zip(a1, a2, s1):
        if x is None:
            continue
        assert torch.equal(x, y)   # run to run
        assert torch.equal(x, z)   # overlapped AdamW == the sweep, over the whole step


@pytest.mark.parametrize("layout", ["cfg5", "groups"])
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_deterministic_overlap_layouts(dev, dtype, deterministic, layout):
    test_deterministic_step_bit_identical(dev, dtype, deterministic, layout)


def test_deterministic_gradients_match_atomic_form(dev):
    """The fixed-order kernels compute the same gradients as the atomic ones up to the rounding of the summation
    order (1e-5 of each tensor's max), on a batch with zero-triple items (the src != i path) and entity / value
    negatives."""
    from k3m_amd import ops
    from k3m_amd.trainer import Trainer
    from k3m_amd.synthetic import synthetic_batch
    from k3m_amd.config import pretrain_config
    from k3m_amd.engine import label_counts
    cfg = pretrain_config(CFG_PATH)
    B = 6
    b = synthetic_batch(cfg, B, dev, seed=71, n_triples=5)
    b["index_p"][1].zero_()   # items 1 and 2 without triples: they reuse item 0's (the bare-except quirk)
    b["index_p"][2].zero_()
    b["_label_counts"] = label_counts(b)
    grads = []
    old = ops.DETERMINISTIC
    try:
        for det in (False, True):
            ops.set_deterministic(det)
            tr = Trainer(cfg, dev, lr=1e-3, warmup_steps=1, total_steps=10, seed=11)
            tr.dropout = False
            out, ctx = tr.engine.forward(b, train=False, seed=0)
            tr.engine.fp.grad.zero_()
            tr.engine.backward(ctx, w_mlm=1.0, w_img=1.0, w_lpm=1.0)
            torch.cuda.synchronize()
            grads.append(tr.engine.fp.grad.clone())
    finally:
        ops.set_deterministic(old)
    fp = tr.engine.fp
    bad = []
    for name, shape in fp.spec:
        o, n = fp.offsets[name], math.prod(shape)
        x, y = grads[0][o:o + n], grads[1][o:o + n]
        # key biases and struc_w2.bias: gradients that are zero up to rounding (a softmax gradient sums to 0)
        tol = 1e-5 * float(x.abs().max()) + 1e-7
        if float((x - y).abs().max()) > tol:
            bad.append((name, float((x - y).abs().max()), tol))
    assert not bad, bad[:10]
    for name in ("embeddings.word_embeddings.weight", "struc_w2.weight", "struc_w1.weight"):
        o = fp.offsets[name]
        assert float(grads[1][o:o + math.prod(dict(fp.spec)[name])].abs().max()) > 0, name
