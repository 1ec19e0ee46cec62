"""The drop-in boundary, driven the way train_concap_struc.py drives the reference:

* imports through the ``vilbert_k3m`` package (train_concap_struc.py:25-26);
* optimizer parameter groups built from ``model.named_parameters()`` (:352-367) and stepped by a
  pytorch_transformers-AdamW optimizer (the oracle's restatement, pytorch_transformers being absent)
  reading ``p.grad``;
* the 10-tuple ``forward`` (:502-524), ``loss = mlm_t + img * w + mlm_pv + lpm`` (:531-533),
  ``loss.backward()`` (:569), ``optimizer.step(); optimizer.zero_grad()`` (:573-574);
* ``state_dict()`` with the reference's 999 keys (:691-705);
* the loaders' iterator contract (dataset:413) feeding the model unchanged.
Checked against the golden vectors recorded from the reference model (losses 1e-3, gradient norms
5e-3, as tests/test_gpu_parity.py)."""
import json
import os

import numpy as np
import pytest
import torch

from golden_util import HERE, load_case, case_config, case_batch, case_noise

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda")


class RefAdamW(torch.optim.Optimizer):
    """pytorch_transformers 1.1.0 AdamW semantics over param groups (oracle restatement)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.98), eps=1e-8, weight_decay=0.0):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self):
        from oracle.k3m_oracle import adamw_step
        for gr in self.param_groups:
            for p in gr["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["m"] = torch.zeros_like(p)
                    st["v"] = torch.zeros_like(p)
                st["step"] += 1
                adamw_step(p.data, p.grad, st["m"], st["v"], st["step"], gr["lr"], gr["weight_decay"],
                           gr["betas"][0], gr["betas"][1], gr["eps"])


def _driver_forward(model, tb, dev, noise, ent, val):
    return model(tb["input_ids"], tb["image_feat"], tb["image_loc"], tb["segment_ids"], tb["input_mask"],
                 tb["image_mask"], tb["lm_label_ids"], tb["image_label"], tb["image_target"], tb["is_next"],
                 output_all_attention_masks=False, input_ids_pv=tb["input_ids_pv"],
                 token_type_ids_pv=tb["segment_ids_pv"], attention_mask_pv=tb["input_mask_pv"],
                 masked_lm_labels_pv=tb["lm_label_ids_pv"], next_sentence_label_pv_v=tb["is_next_pv_v"],
                 next_sentence_label_pv_t=tb["is_next_pv_t"], index_p=tb["index_p"], index_v=tb["index_v"],
                 device=dev, gumbel_noise=noise, ent_neg=ent, val_neg=val)


def test_driver_call_sequence_matches_golden(dev):
    from vilbert_k3m.vilbert_k3m import BertForMultiModalPreTraining_tri_stru
    from k3m_amd.weights import param_values
    g = load_case("bs2_hard")
    cfg = case_config(g)
    model = BertForMultiModalPreTraining_tri_stru(cfg, device=dev)
    vals = param_values(cfg, int(g["weight_seed"]))
    missing = model.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()})
    assert not missing
    model.eval()
    no_decay = ["bias", "LayerNorm.bias", "LayerNorm.weight"]
    param_optimizer = list(model.named_parameters())
    assert len(param_optimizer) == 998
    groups = [{"params": [p for n, p in param_optimizer if not any(nd in n for nd in no_decay)], "weight_decay": 0.01},
              {"params": [p for n, p in param_optimizer if any(nd in n for nd in no_decay)], "weight_decay": 0.0}]
    opt = RefAdamW(groups, lr=1e-4, eps=1e-8, betas=(0.9, 0.98))
    tb = {k: v.to(dev) for k, v in case_batch(g).items()}
    noise = {k: v.to(dev) for k, v in case_noise(g).items()}
    ent, val = torch.from_numpy(g["ent_neg"]), torch.from_numpy(g["val_neg"])
    outs = _driver_forward(model, tb, dev, noise, ent, val)
    assert len(outs) == 10
    mlm_t, img, _, mlm_pv, _, _, nsp, c_init, c_final, lpm = outs
    loss = mlm_t + img * 1.0 + mlm_pv + lpm
    got = np.array([float(x) for x in (mlm_t, img, mlm_pv, lpm, nsp, loss)])
    np.testing.assert_allclose(got, g["losses"], rtol=1e-3, atol=1e-4)
    np.testing.assert_allclose(c_final.detach().cpu().numpy(), g["c_final"], rtol=1e-3, atol=1e-4)
    loss.backward()
    named = dict(model.named_parameters())
    grads = {}
    for n, ref in zip(list(g["grad_norm_names"]), g["grad_norms"]):
        p = named[n]
        gn = 0.0 if p.grad is None else float(p.grad.double().norm())
        if np.isnan(ref):
            assert gn == 0.0, n
        else:
            assert abs(gn - ref) <= 5e-3 * ref + 1e-6, (n, gn, ref)
    for n in ("encoder.layer.0.attention.self.query.weight", "struc_w1.weight", "cls.predictions.bias",
              "encoder.c_layer.2.biattention.key2.bias"):
        grads[n] = named[n].grad.detach().cpu().clone()
    before = {n: named[n].detach().cpu().clone() for n in grads}
    opt.step()
    from oracle.k3m_oracle import adamw_step
    for n in grads:
        p = before[n].clone()
        adamw_step(p, grads[n], torch.zeros_like(p), torch.zeros_like(p), 1, 1e-4,
                   0.0 if any(nd in n for nd in no_decay) else 0.01)
        np.testing.assert_allclose(named[n].detach().cpu().numpy(), p.numpy(), rtol=1e-6, atol=1e-9, err_msg=n)
    opt.zero_grad()
    assert named["struc_w1.weight"].grad is None
    # a second backward after zero_grad(set_to_none) starts from zero gradients (no stale sums)
    outs = _driver_forward(model, tb, dev, noise, ent, val)
    (outs[0] + outs[1] + outs[3] + outs[9]).backward()
    g2 = named["struc_w1.weight"].grad
    assert g2 is not None and torch.isfinite(g2).all()
    sd = model.state_dict()
    inv = json.load(open(os.path.join(HERE, "golden", "param_inventory.json")))   # the reference model's
    assert [n for n, _ in model.named_parameters()] == [n for n, _ in inv["params"]]
    assert len(sd) == 999 and sorted(sd) == sorted([n for n, _ in inv["params"]] + ["cls.predictions.decoder.weight"])
    assert sd["cls.predictions.decoder.weight"].data_ptr() == sd["embeddings.word_embeddings.weight"].data_ptr()


def test_loader_feeds_driver_loop(dev, tmp_path):
    """ConceptCapLoaderTrain_struc with the driver's kwargs (incl. local_rank) on raw product rows:
    the 19-item batches go straight into the model; the head buffers are sized without a sync."""
    from vilbert_k3m.datasets import ConceptCapLoaderTrain_struc
    from vilbert_k3m.vilbert_k3m import BertForMultiModalPreTraining_tri_stru
    from k3m_amd.config import pretrain_config
    from golden_util import CFG_PATH
    from test_data import char_tokenizer
    rows = []
    for i in range(6):
        pv = "#;#".join("p%d%d#:#v%d%d" % (i, j, j, i) for j in range(3 + i))
        rows.append("%d\titem title %d with words\thttp://img/%d.jpg\t%s\tcat" % (1000 + i, i, i, pv))
    (tmp_path / "train.tsv").write_text("\n".join(rows) + "\n", encoding="utf-8")
    loader = ConceptCapLoaderTrain_struc(str(tmp_path), "train.tsv", char_tokenizer(), max_seq_len=36,
                                         max_seq_len_pv=128, max_num_pv=20, max_region_len=36, batch_size=3,
                                         visual_target=0, v_target_size=1601, num_workers=2, local_rank=0,
                                         objective=2, cache=100, serializer=None, seed=1, synthetic_regions=3)
    assert loader.num_dataset == 6 and len(loader) == 2
    cfg = pretrain_config(CFG_PATH)
    model = BertForMultiModalPreTraining_tri_stru(cfg, device=dev)
    model.train()
    n = 0
    for step, batch in enumerate(loader):
        index_p = torch.tensor(batch[-3]).cuda(device=dev, non_blocking=True)
        index_v = torch.tensor(batch[-2]).cuda(device=dev, non_blocking=True)
        batch = tuple(t.cuda(device=dev, non_blocking=True) for t in batch[:-3])
        (input_ids, input_mask, segment_ids, lm_label_ids, is_next, input_ids_pv, input_mask_pv, segment_ids_pv,
         lm_label_ids_pv, is_next_pv_v, is_next_pv_t, image_feat, image_loc, image_target, image_label,
         image_mask) = batch
        assert getattr(lm_label_ids, "_k3m_n_labels", None) is not None     # travels through .cuda()
        outs = model(input_ids, image_feat, image_loc, segment_ids, input_mask, image_mask, lm_label_ids,
                     image_label, image_target, is_next, output_all_attention_masks=False, input_ids_pv=input_ids_pv,
                     token_type_ids_pv=segment_ids_pv, attention_mask_pv=input_mask_pv,
                     masked_lm_labels_pv=lm_label_ids_pv, next_sentence_label_pv_v=is_next_pv_v,
                     next_sentence_label_pv_t=is_next_pv_t, index_p=index_p, index_v=index_v, device=dev)
        loss = outs[0] + outs[1] + outs[3] + outs[9]
        loss.backward()
        assert np.isfinite(float(loss))
        n += 1
    assert n == 2


def test_standin_adamw_state_layout_roundtrip(dev):
    """pytorch_transformers.AdamW stand-in: moments shaped like the parameter (the reference's state_dict
    layout, train_concap_struc.py:293 resume), an odd-sized (1601-element, the image-decoder bias) tensor
    stepped through padded staging, and a state_dict -> load_state_dict round trip that continues exactly."""
    from pytorch_transformers.optimization import AdamW
    from oracle.k3m_oracle import adamw_step
    torch.manual_seed(0)
    shapes = [(1601,), (7, 3), (64, 16)]
    ps = [torch.nn.Parameter(torch.randn(s, device=dev)) for s in shapes]
    grads = [[torch.randn(s, device=dev) for s in shapes] for _ in range(4)]
    ref = [p.detach().cpu().clone() for p in ps]
    rm = [torch.zeros_like(r) for r in ref]
    rv = [torch.zeros_like(r) for r in ref]
    opt = AdamW([{"params": ps, "weight_decay": 0.01}], lr=1e-3, eps=1e-8, betas=(0.9, 0.98))

    def run(o, params, it):
        for p, g in zip(params, grads[it]):
            p.grad = g.clone()
        o.step()

    for it in range(2):
        run(opt, ps, it)
        for i in range(len(ps)):
            adamw_step(ref[i], grads[it][i].cpu(), rm[i], rv[i], it + 1, 1e-3, 0.01, 0.9, 0.98, 1e-8)
    sd = opt.state_dict()
    for i, s in enumerate(shapes):
        st = sd["state"][i]
        assert tuple(st["exp_avg"].shape) == s and tuple(st["exp_avg_sq"].shape) == s and st["step"] == 2
    ps2 = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    opt2 = AdamW([{"params": ps2, "weight_decay": 0.01}], lr=1e-3, eps=1e-8, betas=(0.9, 0.98))
    opt2.load_state_dict(sd)
    for it in range(2, 4):
        run(opt2, ps2, it)
        for i in range(len(ps)):
            adamw_step(ref[i], grads[it][i].cpu(), rm[i], rv[i], it + 1, 1e-3, 0.01, 0.9, 0.98, 1e-8)
    for i in range(len(ps)):
        np.testing.assert_allclose(ps2[i].detach().cpu().numpy(), ref[i].numpy(), rtol=2e-6, atol=1e-7)
        np.testing.assert_allclose(opt2.state[ps2[i]]["exp_avg"].cpu().numpy(), rm[i].numpy(), rtol=2e-6, atol=1e-9)
    bad = torch.nn.Parameter(torch.zeros(1601, device=dev))
    opt3 = AdamW([bad], lr=1e-3)
    opt3.state[bad] = {"step": 1, "exp_avg": torch.zeros(1604, device=dev), "exp_avg_sq": torch.zeros(1604, device=dev)}
    bad.grad = torch.ones_like(bad)
    with pytest.raises(ValueError, match="moments"):
        opt3.step()


def test_half_switches_to_bf16_mode(dev):
    """``model.half()`` (train_concap_struc.py:299-300): same 998 parameters with the same values, now views of
    the 16-bit engine's buffer (bf16 encoder, fp32 master weights); the driver's fp16 inputs (:496-499) are
    accepted; forward / backward run and the losses stay within the bf16 mode's bars of the fp32 model's."""
    from vilbert_k3m.vilbert_k3m import BertForMultiModalPreTraining_tri_stru
    from k3m_amd.weights import param_values
    g = load_case("bs2_hard")
    cfg = case_config(g)
    model = BertForMultiModalPreTraining_tri_stru(cfg, device=dev)
    vals = param_values(cfg, int(g["weight_seed"]))
    model.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()})
    model.eval()
    tb = {k: v.to(dev) for k, v in case_batch(g).items()}
    noise = {k: v.to(dev) for k, v in case_noise(g).items()}
    ent, val = torch.from_numpy(g["ent_neg"]), torch.from_numpy(g["val_neg"])
    ref = [float(x) for x in _driver_forward(model, tb, dev, noise, ent, val)[:2]]
    before = {n: p.detach().clone() for n, p in model.named_parameters()}
    assert model.half() is model and model.engine.dtype == "bf16"
    named = list(model.named_parameters())
    assert [n for n, _ in named] == list(before)
    for n, p in named:
        assert p.dtype == torch.float32 and torch.equal(p.detach(), before[n]), n
        assert p.data_ptr() == model.engine.fp.p[n].data_ptr()
    for k in ("image_feat", "image_loc", "image_target"):
        tb[k] = tb[k].half()
    outs = _driver_forward(model, tb, dev, noise, ent, val)
    got = [float(x) for x in outs[:2]]
    np.testing.assert_allclose(got, ref, rtol=3e-2, atol=1e-3)
    loss = outs[0] + outs[1] + outs[3] + outs[9]
    loss.backward()
    gq = dict(model.named_parameters())["encoder.layer.0.attention.self.query.weight"].grad
    assert gq is not None and torch.isfinite(gq).all() and float(gq.abs().max()) > 0


def test_half_keeps_frozen_parameters(dev):
    """--freeze then --fp16 (train_concap_struc.py:245-257, then model.half() at :300, then the optimizer groups
    from ``value.requires_grad`` at :371): half() keeps each parameter's requires_grad, so an optimizer built the
    driver's way leaves the frozen embeddings / text layers bit-identical after a step while the rest move."""
    from vilbert_k3m.vilbert_k3m import BertForMultiModalPreTraining_tri_stru
    from pytorch_transformers.optimization import AdamW
    from k3m_amd.weights import param_values
    g = load_case("bs2_hard")
    cfg = case_config(g)
    model = BertForMultiModalPreTraining_tri_stru(cfg, device=dev)
    vals = param_values(cfg, int(g["weight_seed"]))
    model.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()})
    freeze = 1   # the driver's --freeze 1: embeddings and text layers 0..1

    def frozen(n):
        return "embeddings" in n or (n.startswith("encoder.layer.") and int(n.split(".")[2]) <= freeze)
    for n, p in model.named_parameters():
        if frozen(n):
            p.requires_grad = False
    model.half()
    named = list(model.named_parameters())
    assert any(frozen(n) for n, _ in named)
    for n, p in named:
        assert p.requires_grad == (not frozen(n)), n
    before = {n: p.detach().clone() for n, p in named}
    opt = AdamW([p for _, p in named if p.requires_grad], lr=1e-3, eps=1e-8, betas=(0.9, 0.98))
    model.train()
    tb = {k: v.to(dev) for k, v in case_batch(g).items()}
    noise = {k: v.to(dev) for k, v in case_noise(g).items()}
    ent, val = torch.from_numpy(g["ent_neg"]), torch.from_numpy(g["val_neg"])
    outs = _driver_forward(model, tb, dev, noise, ent, val)
    (outs[0] + outs[1] + outs[3] + outs[9]).backward()
    opt.step()
    moved = 0
    for n, p in model.named_parameters():
        if frozen(n):
            assert torch.equal(p.detach(), before[n]), n
        elif not torch.equal(p.detach(), before[n]):
            moved += 1
    assert moved > 100


def test_unequal_mlm_loss_weights(dev):
    """A caller's  a*mlm_t + b*mlm_pv  (the reference sums them with weight 1, train_concap_struc.py:531-533): the
    shared decoder's text and PV gradient rows take their own upstream weights (k3m_scale_rows_by_slot), so the
    gradient equals a * grad(mlm_t) + b * grad(mlm_pv), to the backward's float-atomics rounding."""
    from vilbert_k3m.vilbert_k3m import BertForMultiModalPreTraining_tri_stru
    from k3m_amd.weights import param_values
    g = load_case("bs2_hard")
    cfg = case_config(g)
    model = BertForMultiModalPreTraining_tri_stru(cfg, device=dev)
    vals = param_values(cfg, int(g["weight_seed"]))
    model.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()})
    model.eval()
    tb = {k: v.to(dev) for k, v in case_batch(g).items()}
    noise = {k: v.to(dev) for k, v in case_noise(g).items()}
    ent, val = torch.from_numpy(g["ent_neg"]), torch.from_numpy(g["val_neg"])
    names = ("cls.predictions.bias", "cls.predictions.transform.dense.weight", "embeddings.word_embeddings.weight",
             "encoder.layer.11.output.dense.weight", "encoder.layer.0.attention.self.query.weight")

    def grads(wt, wpv):
        model.zero_grad(set_to_none=True)
        outs = _driver_forward(model, tb, dev, noise, ent, val)
        (wt * outs[0] + wpv * outs[3]).backward()
        named = dict(model.named_parameters())
        return {n: named[n].grad.detach().double().clone() for n in names}
    a, b = 0.7, 1.3
    both = grads(a, b)
    gt = grads(1.0, 0.0)
    gp = grads(0.0, 1.0)
    for n in names:
        ref = a * gt[n] + b * gp[n]
        err = float((both[n] - ref).norm())
        assert err <= 1e-5 * float(ref.norm()) + 1e-9, (n, err, float(ref.norm()))
