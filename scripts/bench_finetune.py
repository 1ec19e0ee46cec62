"""Measure the item-alignment fine-tuning step at the reference run script's
configuration (run_finetune_item_alignment.sh: train_batch_size 32 pairs on one GPU, max_seq_length
50, max_seq_length_pv 256, max_num_pv 30, 36 regions, loss_type ce, if_pre_sampling 1), fp32:
forward of both items as one stacked batch, pair head, backward, torch.optim.AdamW, schedule.

Prints one JSON line (same fields as bench.py): value = pairs/s; roofline of the dominant kernel
(the text-layer FFN1 GEMM over the stacked rows, timed with HIP events on its stream); cpu_baseline
= the CPU oracle on a bounded sample.  Usage: python scripts/bench_finetune.py [--steps 10]
"""
import argparse
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
import bench  # noqa: E402


def pair_batch(cfg, B, dev, seed, T, P, npv, triples):
    from k3m_amd.synthetic import synthetic_batch
    items = [synthetic_batch(cfg, B, dev, seed=seed + k, T=T, P=P, n_triples=triples, npv=npv) for k in (0, 1)]
    names = [("input_ids", "input_ids"), ("token_type_ids", "segment_ids"), ("attention_mask", "input_mask"),
             ("input_ids_pv", "input_ids_pv"), ("token_type_ids_pv", "segment_ids_pv"),
             ("attention_mask_pv", "input_mask_pv"), ("index_p", "index_p"), ("index_v", "index_v"),
             ("image_feat", "image_feat"), ("image_loc", "image_loc"), ("image_attention_mask", "image_mask")]
    pair = {"labels": (torch.arange(B, device=dev) % 2).float()}
    for k, it in ((1, items[0]), (2, items[1])):
        for a, b in names:
            pair["%s_%d" % (a, k)] = it[b]
    return pair


def cpu_baseline(cfg, T, P, npv, triples, steps):
    from oracle import k3m_oracle as O
    from k3m_amd.params import is_frozen, is_no_decay
    from k3m_amd.weights import init_values
    ncores = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(os.cpu_count() or 1, 16)
    torch.set_num_threads(ncores)
    Pm = {k: torch.from_numpy(v).requires_grad_(True) for k, v in init_values(cfg, 0).items()}
    from k3m_amd.synthetic import synthetic_noise
    pair = pair_batch(cfg, 1, "cpu", 7, T, P, npv, triples)
    noise = [synthetic_noise(cfg, 1, seed=s, T=T, P=P) for s in (1, 2)]
    st = {k: (torch.zeros_like(v), torch.zeros_like(v)) for k, v in Pm.items()}

    def step(t):
        _, _, _, loss = O.item_alignment_forward(Pm, cfg, pair, noise[0], noise[1])
        loss.backward()
        with torch.no_grad():
            for k, p in Pm.items():
                if p.grad is None or is_frozen(k):
                    continue
                m, v = st[k]
                O.adamw_torch_step(p.data, p.grad, m, v, t, 5e-5, 0.0 if is_no_decay(k) else 0.01)
                p.grad = None

    step(1)
    t0 = time.perf_counter()
    for t in range(steps):
        step(t + 2)
    dt = time.perf_counter() - t0
    return {"value": round(steps / dt, 4), "unit": "pairs/s", "cores": ncores, "kind": "port",
            "sample": "oracle item_alignment_forward+backward+torch AdamW, fp32, 1 pair, %d timed steps, %.1f s"
                      % (steps, dt)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    a = ap.parse_args()
    from k3m_amd.config import finetune_config
    from k3m_amd.finetune import ItemAlignmentTrainer
    T, P, NPV, TRIPLES = 50, 256, 30, 30
    cfg = finetune_config(os.path.join(HERE, "configs", "bert_base_6layer_6conect.json"), loss_type="ce")
    dev = torch.device("cuda", 0)
    B = a.batch
    tr = ItemAlignmentTrainer(cfg, dev, lr=5e-5, warmup_steps=max(1, (a.steps + a.warmup) // 3),
                              total_steps=10 * (a.steps + a.warmup), seed=42)
    pair = pair_batch(cfg, B, dev, 1234, T, P, NPV, TRIPLES)
    probe = bench.GemmProbe(2 * (2 * B) * T + 2 * (2 * B) * P, cfg.intermediate_size, cfg.hidden_size)
    probe.install()
    for _ in range(a.warmup):
        tr.step(pair)
    torch.cuda.synchronize()
    probe.active = True
    t0 = time.perf_counter()
    for _ in range(a.steps):
        out = tr.step(pair)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    probe.active = False
    gemm_ms = probe.mean_ms()
    Mg, Ng, Kg = probe.key
    achieved = 2.0 * Mg * Ng * Kg / (gemm_ms * 1e-3) if gemm_ms else None
    peak = bench.PEAK_F32_X6
    res = {"metric": "item-alignment fine-tune pairs/sec (bert_base_6layer_6conect, 32 pairs/GPU)",
           "value": round(B * a.steps / dt, 3), "unit": "pairs/s", "n_gpus": 1, "steps": a.steps,
           "warmup": a.warmup, "ms_per_step": round(1000 * dt / a.steps, 3), "higher_is_better": True,
           "vs_baseline": None, "dtype": "fp32", "data": "synthetic pairs (random ids, 36x2048 region feats, 30 triples)",
           "config": {"workload": "K3MForItemAlignment ce, T=50 P=256 NPV=30 R=37, both items stacked (64 items)",
                      "batch_pairs": B},
           "loss": round(float(out["loss"]), 4),
           "roofline": {"bound": "mfma", "kernel": "gemm_x6_kernel text-layer FFN1 %dx%dx%d" % (Mg, Ng, Kg),
                        "achieved": round(achieved / 1e12, 2) if achieved else None, "peak": peak / 1e12,
                        "unit": "TFLOP/s", "frac": round(achieved / peak, 4) if achieved else None,
                        "avg_launch_ms": round(gemm_ms, 4) if gemm_ms else None, "launches": len(probe.events),
                        "traffic": None}}
    if not a.no_cpu_baseline:
        try:
            res["cpu_baseline"] = cpu_baseline(cfg, T, P, NPV, TRIPLES, a.cpu_steps)
        except Exception as e:  # baseline only
            res["cpu_baseline"] = {"error": repr(e)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
