"""Error distribution of the bf16 encoder's logits against the reference's fp32 golden logits (tests/golden,
make_golden.py), per case: the per-element error d = |bf16 - ref| / (row max |ref|) of the 256 recorded MLM
vocabulary columns and of the masked-region logits, its quantiles, the per-column mean over the rows (a
systematic error in a few columns shows there, not in the global mean) and the logsumexp error.  Writes
the JSON the bf16 logit bars of tests/test_gpu_parity.py are set from (profiles/r4_bf16_logit_errors.json).
usage: python scripts/bf16_logit_errors.py out.json"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from golden_util import CASES, load_case, case_config, case_batch, case_noise  # noqa: E402


def stats(d):
    q = np.quantile(d, [0.5, 0.9, 0.99, 0.999])
    return {"n": int(d.size), "mean": float(d.mean()), "p50": float(q[0]), "p90": float(q[1]), "p99": float(q[2]),
            "p999": float(q[3]), "max": float(d.max())}


def main(out):
    from k3m_amd.engine import K3MEngine
    from k3m_amd.weights import param_values
    dev = torch.device("cuda")
    res = {}
    for case in CASES:
        g = load_case(case)
        cfg = case_config(g)
        eng = K3MEngine(cfg, dev, dtype="bf16")
        eng.fp.load(param_values(cfg, int(g["weight_seed"])))
        eng.capture_logits = True
        batch = {k: v.to(dev) for k, v in case_batch(g).items()}
        noise = {k: v.to(dev) for k, v in case_noise(g).items()}
        o, _ = eng.forward(batch, train=False, noise=noise, ent_neg=torch.from_numpy(g["ent_neg"]),
                           val_neg=torch.from_numpy(g["val_neg"]))
        torch.cuda.synchronize()
        mlm = o["mlm_logits"].double().cpu().numpy()
        img = o["img_logits"].double().cpu().numpy()
        ref = g["logit/mlm_rows"].astype(np.float64)
        d = np.abs(mlm[:, g["logit/mlm_cols"]] - ref) / (np.abs(ref).max(1, keepdims=True) + 1e-6)
        refv = g["logit/img_rows"].astype(np.float64)
        dv = np.abs(img - refv) / (np.abs(refv).max(1, keepdims=True) + 1e-6)
        m = mlm.max(1)
        lse = m + np.log(np.exp(mlm - m[:, None]).sum(1))
        res[case] = {"mlm": stats(d), "mlm_col_mean_max": float(d.mean(0).max()),
                     "img": stats(dv), "img_col_mean_max": float(dv.mean(0).max()),
                     "lse_abs_max": float(np.abs(lse - g["logit/mlm_lse"]).max())}
        print(case, json.dumps(res[case]), flush=True)
        del eng
        torch.cuda.empty_cache()
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1])
