"""Item-alignment fine-tuning on the GPU: K3MForItemAlignment through
libk3m_hip against golden vectors recorded from the reference K3MForItemAlignment
(tests/golden/make_finetune_golden.py), eval mode with explicit gumbel noise; the pair collation
kernel against the reference's K3MDataLoader collation; one ItemAlignmentTrainer step against the
CPU oracle + torch.optim.AdamW restatement.  Tolerances as the pretraining parity (1e-3 relative)."""
import os

import numpy as np
import pytest
import torch

from golden_util import FT_CASES, ft_config, ft_noise, ft_pair, load_ft_case

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda")


@pytest.mark.parametrize("case", FT_CASES)
def test_item_alignment_matches_reference_golden(dev, case):
    from k3m_amd.finetune import ARG_NAMES, K3MForItemAlignment
    from k3m_amd.weights import param_values
    g = load_ft_case(case)
    cfg = ft_config(g)
    model = K3MForItemAlignment(cfg, dev)
    model.engine.fp.load(param_values(cfg, int(g["weight_seed"])))
    pair = {k: v.to(dev) for k, v in ft_pair(g).items()}
    n1, n2 = ft_noise(g)
    noise = ({k: v.to(dev) for k, v in n1.items()}, {k: v.to(dev) for k, v in n2.items()})
    e1, e2, probs, loss = model(*[pair[k] for k in ARG_NAMES], train=False, noise=noise)
    model.backward()
    torch.cuda.synchronize()
    np.testing.assert_allclose(float(loss), float(g["out/loss"]), rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(e1.cpu().numpy(), g["out/e1"], rtol=1e-3, atol=1e-4)
    np.testing.assert_allclose(e2.cpu().numpy(), g["out/e2"], rtol=1e-3, atol=1e-4)
    np.testing.assert_allclose(probs.cpu().numpy(), g["out/probs"], rtol=1e-3, atol=1e-5)
    G = model.engine.fp.g
    for k in g:
        if k.startswith("grad_full/"):
            n = k.split("/", 1)[1]
            ref = g[k]
            err = np.abs(G[n].cpu().numpy() - ref).max()
            assert err <= 5e-3 * np.abs(ref).max() + 1e-6, (n, err, np.abs(ref).max())
    for n, ref in zip(list(g["grad_norm_names"]), g["grad_norms"]):
        gn = float(G[n].double().norm())
        if np.isnan(ref):
            assert gn == 0.0, n
        else:
            assert abs(gn - ref) <= 5e-3 * ref + 1e-6, (n, gn, ref)


def test_pair_collator_matches_reference(dev):
    from k3m_amd import data as D
    from tests.test_data import ft_preprocessor, ft_records
    z = np.load(os.path.join(HERE, "golden", "golden_ft_data.npz"))
    g = {k: z[k] for k in z.files}
    pre = ft_preprocessor(g)
    prepared = [pre.prepare(r) for r in ft_records(g)]
    col = D.PairCollator(dev, pre.max_region_len, pre.v_feature_size, pre.v_target_size)
    out, ids1, ids2 = col(prepared)
    torch.cuda.synchronize()
    assert np.array_equal(out["labels"].cpu().numpy(), g["out/labels"])
    for k in (1, 2):
        assert np.array_equal(out["image_feat_%d" % k].cpu().numpy(), g["out/coll_image_feat_%d" % k], equal_nan=True)
        assert np.array_equal(out["image_loc_%d" % k].cpu().numpy(), g["out/coll_image_loc_%d" % k])
        assert np.array_equal(out["image_attention_mask_%d" % k].cpu().numpy(), g["out/coll_image_mask_%d" % k])
        for a, b in (("input_ids", "input_ids"), ("attention_mask", "input_mask"), ("token_type_ids", "segment_ids"),
                     ("input_ids_pv", "input_ids_pv"), ("attention_mask_pv", "input_mask_pv"), ("index_p", "index_p"),
                     ("index_v", "index_v"), ("image_target", "image_target")):
            assert np.array_equal(out["%s_%d" % (a, k)].cpu().numpy(), g["out/%s_%d" % (b, k)]), (a, k)


def test_trainer_step_matches_oracle(dev):
    """One ItemAlignmentTrainer step (dropout probabilities 0, explicit noise): the gradients
    against the CPU oracle (relative to each tensor's scale), then the torch.optim.AdamW update of
    k3m_adamw_torch against the oracle's restatement applied to the same gradients."""
    from k3m_amd.finetune import ARG_NAMES, ItemAlignmentTrainer
    from k3m_amd.params import is_frozen, is_no_decay
    from k3m_amd.weights import param_values
    from oracle import k3m_oracle as O
    g = load_ft_case("ce")
    cfg = ft_config(g)
    cfg.hidden_dropout_prob = cfg.attention_probs_dropout_prob = 0.0
    cfg.v_hidden_dropout_prob = cfg.v_attention_probs_dropout_prob = 0.0
    lr = 1e-4
    tr = ItemAlignmentTrainer(cfg, dev, lr=lr, warmup_steps=0, total_steps=100, init=False)
    vals = param_values(cfg, int(g["weight_seed"]))
    tr.engine.fp.load(vals)
    pair = {k: v.to(dev) for k, v in ft_pair(g).items()}
    n1, n2 = ft_noise(g)
    _, _, _, loss = tr.model.forward(*[pair[k] for k in ARG_NAMES], train=True,
                                     noise=({k: v.to(dev) for k, v in n1.items()}, {k: v.to(dev) for k, v in n2.items()}))
    tr.model.backward()
    torch.cuda.synchronize()
    G = {n: t.cpu().clone() for n, t in tr.engine.fp.g.items()}
    tr.optimizer_step()
    torch.cuda.synchronize()
    torch.set_num_threads(16)
    P = {k: torch.from_numpy(v).requires_grad_(True) for k, v in vals.items()}
    _, _, _, ref_loss = O.item_alignment_forward(P, cfg, ft_pair(g), n1, n2)
    ref_loss.backward()
    np.testing.assert_allclose(float(loss), float(ref_loss), rtol=1e-3)
    for n in ["classifier.out_proj.weight", "classifier.dense.weight", "struc_w1.weight", "encoder.layer.0.output.dense.bias",
              "v_embeddings.image_embeddings.weight", "embeddings.LayerNorm.weight", "t_pooler.dense.weight"]:
        ref = P[n].grad
        if ref is None:
            assert is_frozen(n) and float(G[n].abs().max()) == 0.0, n
        else:
            err = (G[n] - ref).abs().max().item()
            assert err <= 5e-3 * ref.abs().max().item() + 1e-6, (n, err)
        p = torch.from_numpy(vals[n]).clone()
        if not is_frozen(n):
            m, v = torch.zeros_like(p), torch.zeros_like(p)
            O.adamw_torch_step(p, G[n], m, v, 1, lr, 0.0 if is_no_decay(n) else 0.01)
        got = tr.engine.fp.p[n].cpu()
        np.testing.assert_allclose(got.numpy(), p.numpy(), rtol=1e-6, atol=1e-7 * lr / 1e-4, err_msg=n)


def test_evaluate_and_save(dev, tmp_path):
    """evaluate() runs the eval loop of finetune.py (precision/recall/F1 per threshold over several
    batches) and save_model() writes the 989-key state_dict the reference saves per epoch."""
    from k3m_amd.finetune import K3MForItemAlignment, evaluate, save_model
    from k3m_amd.weights import param_values
    g = load_ft_case("ce")
    cfg = ft_config(g)
    model = K3MForItemAlignment(cfg, dev)
    model.engine.fp.load(param_values(cfg, int(g["weight_seed"])))
    pair = {k: v.to(dev) for k, v in ft_pair(g).items()}
    metrics, probs, labels = evaluate(model, [pair, pair])
    assert len(metrics) == 9 and probs.shape == (4,) and labels.shape == (4,)
    assert all(0.0 <= m["f1"] <= 1.0 for m in metrics)
    path = str(tmp_path / "K3M_item_alignment-1_epoch-0.bin")
    save_model(model, path)
    sd = torch.load(path, map_location="cpu", weights_only=True)
    assert len(sd) == 989 and "classifier.out_proj.weight" in sd
