"""Hard gumbel-gate flip rates at full size (SURVEY §7 "report the tie rate").

The hard gate (vilbert_k3m.py:2363-2372) picks, per (row, channel), the argmax of three gate logits plus gumbel
noise.  Two computations of the same step that differ only in rounding pick different sources where two of those
values are within the rounding difference of a tie.  This script runs the same eval-mode forward twice and counts
the choices that differ:
  * config 2 shapes (fp32): the bf16x6 GEMMs against the exact-f32 MFMA GEMMs;
  * configs 3, 4, 5 shapes: the bf16 encoder against the fp32 one.
Same weights (param_values), batch, gumbel noise and negatives for both runs.  Writes one JSON file.

    python scripts/gate_flips.py [out.json]
"""
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

from k3m_amd import ops, _lib as L                       # noqa: E402
from k3m_amd.config import pretrain_config               # noqa: E402
from k3m_amd.engine import K3MEngine                     # noqa: E402
from k3m_amd.synthetic import synthetic_batch, synthetic_noise   # noqa: E402
from k3m_amd.weights import param_values                 # noqa: E402

LOSSES = ("masked_lm_loss", "masked_img_loss", "masked_lm_loss_pv", "loss_lpm", "next_sentence_loss", "loss")
SHAPES = {2: dict(B=64, T=36, P=128, nbox=36, n_triples=10, npv=20),
          3: dict(B=64, T=36, P=128, nbox=36, n_triples=10, npv=20),
          4: dict(B=256, T=128, P=128, nbox=100, n_triples=10, npv=20),
          5: dict(B=128, T=36, P=320, nbox=36, n_triples=50, npv=50)}


def tables(B, NPV, n):
    ent = torch.full((B, NPV, 2), -1, dtype=torch.int64)
    val = torch.full((B, NPV, 2), -1, dtype=torch.int64)
    for i in range(B):
        for j in range(n):
            ent[i, j, 0], ent[i, j, 1] = (i + 1) % B, (i + 5) % B
            val[i, j, 0], val[i, j, 1] = (j + 1) % n, (j + 2) % n
    return ent, val


def run(cfg, dev, vals, inp, dtype, algo):
    batch, noise, ent, val = inp
    old = ops.F32_ALGO
    ops.F32_ALGO = algo
    try:
        eng = K3MEngine(cfg, dev, dtype=dtype)
        eng.fp.load(vals)
        out, ctx = eng.forward(batch, train=False, noise=noise, ent_neg=ent, val_neg=val)
        torch.cuda.synchronize()
    finally:
        ops.F32_ALGO = old
    fus = ctx["fus"][0]
    gates = {m: fus[m][3].detach().cpu().numpy() for m in ("v", "t", "pv")}
    losses = [float(out[k]) for k in LOSSES]
    del eng, out, ctx
    torch.cuda.empty_cache()
    return gates, losses


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "gpurun_out", "gate_flip_rate.json")
    dev = torch.device("cuda")
    cfg = pretrain_config(os.path.join(HERE, "configs", "bert_base_6layer_6conect.json"))
    vals = param_values(cfg, 17)
    rec = {"what": __doc__.strip().splitlines()[0], "rows": []}
    for c in (2, 3, 4, 5):
        s = SHAPES[c]
        B = s["B"]
        t0 = time.time()
        batch = {k: v.to(dev) for k, v in synthetic_batch(cfg, B, "cpu", seed=31, T=s["T"], P=s["P"], n_boxes=s["nbox"],
                                                             n_triples=s["n_triples"], npv=s["npv"]).items()}
        noise = {k: v.to(dev) for k, v in synthetic_noise(cfg, B, seed=32, T=s["T"], P=s["P"], R=s["nbox"] + 1).items()}
        ent, val = tables(B, batch["index_p"].shape[1], s["n_triples"] - 1)
        inp = (batch, noise, ent, val)
        if c == 2:
            a, b = ("fp32", L.F32_SPLIT_BF16X6), ("fp32", L.F32_MFMA_F32)
            pair = "fp32 bf16x6 GEMMs vs exact-f32 MFMA GEMMs"
        else:
            a, b = ("bf16", L.F32_SPLIT_BF16X6), ("fp32", L.F32_SPLIT_BF16X6)
            pair = "bf16 encoder vs fp32 encoder"
        ga, la = run(cfg, dev, vals, inp, *a)
        gb, lb = run(cfg, dev, vals, inp, *b)
        row = {"config": c, "pair": pair, "B": B, "T": s["T"], "P": s["P"], "R": s["nbox"] + 1}
        nd = nt = 0
        for m in ("v", "t", "pv"):
            d = int((ga[m] != gb[m]).sum())
            row["flips_" + m] = d
            row["choices_" + m] = int(ga[m].size)
            row["rate_" + m] = d / ga[m].size
            nd, nt = nd + d, nt + ga[m].size
        row["flips"], row["choices"], row["rate"] = nd, int(nt), nd / nt
        row["loss_rel"] = [abs(x - y) / max(abs(y), 1e-3) for x, y in zip(la, lb)]
        row["seconds"] = round(time.time() - t0, 1)
        rec["rows"].append(row)
        print(json.dumps(row), flush=True)
        del batch, noise, inp
        torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(os.path.abspath(out_path)), exist_ok=True)
    with open(out_path, "w") as f:
        json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
