"""Pin the CPU oracle against golden vectors recorded from the reference model itself
(tests/golden/make_golden.py).  Full-size bert_base_6layer_6conect, bs=2/3, eval mode."""
import numpy as np
import pytest
import torch

from golden_util import CASES, load_case, case_config, case_batch, case_noise, check_logits, check_img_logits


@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_reference(case):
    from oracle import k3m_oracle as O
    from k3m_amd.weights import param_values
    g = load_case(case)
    cfg = case_config(g)
    torch.set_num_threads(8)
    P = {k: torch.from_numpy(v).requires_grad_(True) for k, v in param_values(cfg, int(g["weight_seed"])).items()}
    out = O.forward(P, cfg, case_batch(g), case_noise(g), torch.from_numpy(g["ent_neg"]), torch.from_numpy(g["val_neg"]))
    out["loss"].backward()
    got = np.array([float(out[k].detach()) for k in ("masked_lm_loss", "masked_img_loss", "masked_lm_loss_pv", "loss_lpm",
                                           "next_sentence_loss", "loss")])
    np.testing.assert_allclose(got, g["losses"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(out["c_initial"].detach().numpy(), g["c_initial"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(out["c_final"].detach().numpy(), g["c_final"], rtol=1e-4, atol=1e-5)
    b = case_batch(g)
    V = out["logits_t"].shape[-1]
    rows = torch.cat([out["logits_t"].reshape(-1, V)[b["lm_label_ids"].reshape(-1) != -1],
                      out["logits_pv"].reshape(-1, V)[b["lm_label_ids_pv"].reshape(-1) != -1]]).detach()
    check_logits(g, rows.numpy(), g["logit/img_rows"], 1e-5, case)
    lv = out["logits_v"].detach()
    lv = lv[:, 1:] if lv.shape[1] == b["image_label"].shape[1] + 1 else lv
    check_img_logits(g, lv.reshape(-1, lv.shape[-1])[b["image_label"].reshape(-1) == 1].numpy(), 1e-5, case)
    for k in g:
        if k.startswith("grad_full/") or k.startswith("grad_slice/"):
            n = k.split("/", 1)[1]
            gr = P[n].grad
            gr = torch.zeros_like(P[n]) if gr is None else gr
            if k.startswith("grad_slice/"):
                gr = gr[:4] if gr.dim() == 2 else gr[:256]
            np.testing.assert_allclose(gr.numpy(), g[k], rtol=2e-3, atol=2e-6, err_msg=n)
    names = list(g["grad_norm_names"])
    for n, ref in zip(names, g["grad_norms"]):
        gr = P[n].grad
        if np.isnan(ref):
            assert gr is None or float(gr.abs().max()) == 0.0, n
        else:
            assert gr is not None, n
            np.testing.assert_allclose(float(gr.double().norm()), ref, rtol=1e-3, atol=1e-7, err_msg=n)
