"""Item-alignment fine-tuning on the CPU: the parameter inventory and the
CPU oracle against golden vectors recorded from the reference K3MForItemAlignment itself
(tests/golden/make_finetune_golden.py), plus the torch.optim.AdamW restatement."""
import json
import os

import numpy as np
import pytest
import torch

from golden_util import FT_CASES, HERE, ft_config, ft_noise, ft_pair, load_ft_case


@pytest.mark.parametrize("loss_type", ["ce", "cosine"])
def test_finetune_inventory_matches_reference(loss_type):
    from k3m_amd.config import finetune_config
    from k3m_amd.params import param_spec
    from golden_util import CFG_PATH
    inv = json.load(open(os.path.join(HERE, "golden", "param_inventory_finetune.json")))
    cfg = finetune_config(CFG_PATH, loss_type=loss_type)
    got = [[n, list(s)] for n, s in param_spec(cfg)]
    assert got == inv[loss_type]
    assert [n for n, _ in got] == inv[loss_type + "_state_dict_keys"]   # no tied weights in this model


@pytest.mark.parametrize("case", FT_CASES)
def test_finetune_oracle_matches_reference(case):
    from oracle import k3m_oracle as O
    from k3m_amd.weights import param_values
    g = load_ft_case(case)
    cfg = ft_config(g)
    torch.set_num_threads(8)
    P = {k: torch.from_numpy(v).requires_grad_(True) for k, v in param_values(cfg, int(g["weight_seed"])).items()}
    n1, n2 = ft_noise(g)
    e1, e2, probs, loss = O.item_alignment_forward(P, cfg, ft_pair(g), n1, n2)
    loss.backward()
    np.testing.assert_allclose(float(loss), float(g["out/loss"]), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(e1.detach().numpy(), g["out/e1"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(e2.detach().numpy(), g["out/e2"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(probs.detach().numpy(), g["out/probs"], rtol=1e-5, atol=1e-6)
    for k in g:
        if k.startswith("grad_full/"):
            n = k.split("/", 1)[1]
            gr = P[n].grad
            gr = torch.zeros_like(P[n]) if gr is None else gr
            np.testing.assert_allclose(gr.numpy(), g[k], rtol=2e-3, atol=2e-6, err_msg=n)
    for n, ref in zip(list(g["grad_norm_names"]), g["grad_norms"]):
        gr = P[n].grad
        if np.isnan(ref):
            assert gr is None or float(gr.abs().max()) == 0.0, n
        else:
            assert gr is not None, n
            np.testing.assert_allclose(float(gr.double().norm()), ref, rtol=1e-3, atol=1e-7, err_msg=n)


def test_adamw_torch_restatement_matches_torch():
    from oracle import k3m_oracle as O
    torch.manual_seed(0)
    p0 = torch.randn(1000)
    p = torch.nn.Parameter(p0.clone())
    opt = torch.optim.AdamW([p], lr=5e-3, betas=(0.9, 0.98), eps=1e-8, weight_decay=0.01, foreach=False)
    q, m, v = p0.clone(), torch.zeros(1000), torch.zeros(1000)
    for step in range(1, 6):
        g = torch.randn(1000)
        p.grad = g.clone()
        opt.step()
        O.adamw_torch_step(q, g, m, v, step, 5e-3, 0.01)
    np.testing.assert_allclose(q.numpy(), p.detach().numpy(), rtol=1e-6, atol=1e-7)
