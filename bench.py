"""Benchmark: K3M tri-modal pretraining step (bert_base_6layer_6conect) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 64] [--no-cpu-baseline]

One step = forward + backward + (RCCL gradient all-reduce when N > 1) + AdamW + LR schedule over
one synthetic batch resident in HBM (SURVEY.md §8(d) input spec; random token ids, 36x2048 region
features, 10 PV triples).  N > 1: launched by torch.distributed.run, one rank per GPU, each rank
processes its own bs=64 batch (weak scaling, global batch = 64 N).

Prints ONE JSON line (rank 0) with the driver's contract plus
  roofline     — the dominant kernel (the fp32 MFMA GEMM of the text-layer FFN, timed with HIP
                 events on its stream over the timed steps) against the f32 MFMA peak;
  cpu_baseline — the CPU oracle (plain PyTorch fp32 restatement of the same step, oracle/) timed
                 on the host cores on a bounded sample (rank 0, N = 1 only).
"""
import argparse
import json
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

PEAK_F32_MFMA = 157.3e12      # MI355X f32 MFMA dense peak (MI355X_MICROARCH.md)
PEAK_BF16_MFMA = 2.5e15
PEAK_F32_X6 = PEAK_BF16_MFMA / 6   # fp32 GEMM as 6 bf16 MFMA partial products (gemm_x6_tile.h)
REF_FLOPS_PER_SAMPLE = 319.31e9   # reference algorithmic fwd+bwd FLOPs/sample at config 2


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"],
                    help="fp32: configs[1] (the metric's config); bf16: mixed-precision encoder (configs[2])")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-batch", type=int, default=2)
    ap.add_argument("--cpu-steps", type=int, default=10)
    ap.add_argument("--backend", default="nccl", help="nccl (RCCL) for real runs; gloo only to rehearse the "
                    "multi-rank path with several ranks sharing one GPU")
    return ap.parse_args()


class GemmProbe(object):
    """Times every launch of one GEMM shape with HIP events on the launching stream."""

    def __init__(self, m, n, k):
        self.key = (m, n, k)
        self.events = []
        self.active = False

    def install(self):
        from k3m_amd import ops
        orig = ops.gemm
        probe = self

        def wrapped(a, a_trans, b, b_trans, c, m, n, k, *args, **kw):
            if probe.active and (m, n, k) == probe.key and ops._grouper is None:   # a deferred GEMM is not timed here
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                r = orig(a, a_trans, b, b_trans, c, m, n, k, *args, **kw)
                e.record()
                probe.events.append((s, e))
                return r
            return orig(a, a_trans, b, b_trans, c, m, n, k, *args, **kw)

        ops.gemm = wrapped

    def mean_ms(self):
        if not self.events:
            return None
        return sum(s.elapsed_time(e) for s, e in self.events) / len(self.events)


def pmc_traffic(key, kernel_prefix):
    """HBM-side bytes per launch of the probed GEMM, from the committed rocprofv3 PMC passes
    (profiles/r1_gemm_ffn1_pmc.json: FETCH_SIZE x2 gfx950 correction + WRITE_SIZE), or None."""
    path = os.path.join(HERE, "profiles", "r1_gemm_ffn1_pmc.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if tuple(d.get("shape", ())) != tuple(key) or kernel_prefix not in d.get("kernel", ""):
        return None
    return int(d["traffic_bytes"])


def cpu_baseline(cfg, bsz, steps):
    """Oracle (torch CPU fp32) fwd+bwd+AdamW on a bounded sample; baseline only."""
    from oracle import k3m_oracle as O
    from k3m_amd.weights import init_values
    from k3m_amd.synthetic import synthetic_batch, synthetic_noise
    ncores = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(os.cpu_count() or 1, 16)
    torch.set_num_threads(ncores)
    P = {k: torch.from_numpy(v).requires_grad_(True) for k, v in init_values(cfg, 0).items()}
    batch = synthetic_batch(cfg, bsz, "cpu", seed=99)
    noise = synthetic_noise(cfg, bsz, seed=1)
    NPV = batch["index_p"].shape[1]
    ent = torch.full((bsz, NPV, 2), -1, dtype=torch.int64)
    val = torch.full((bsz, NPV, 2), -1, dtype=torch.int64)
    for i in range(bsz):
        for j in range(10):
            ent[i, j, 0] = (i + 1) % bsz if bsz > 1 else -1
            val[i, j, 0] = (j + 1) % 10
    state = {k: (torch.zeros_like(v), torch.zeros_like(v)) for k, v in P.items()}

    def step(t):
        out = O.forward(P, cfg, batch, noise, ent, val)
        out["loss"].backward()
        with torch.no_grad():
            for k, p in P.items():
                if p.grad is None:
                    continue
                m, v = state[k]
                O.adamw_step(p.data, p.grad, m, v, t, 1e-4, 0.0 if ("bias" in k or "LayerNorm" in k) else 0.01)
                p.grad = None

    step(1)
    t0 = time.perf_counter()
    for t in range(steps):
        step(t + 2)
    dt = time.perf_counter() - t0
    return {"value": round(bsz * steps / dt, 4), "unit": "samples/s", "cores": ncores, "kind": "port",
            "sample": "oracle/k3m_oracle.py fwd+bwd+AdamW, fp32, bs=%d, %d timed steps after 1 warm-up, "
                      "%.1f s" % (bsz, steps, dt)}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    ddp = None
    if world > 1:
        import torch.distributed as dist
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)
        from k3m_amd.ddp import GradAllReducer
    from k3m_amd.config import pretrain_config
    from k3m_amd.trainer import Trainer
    from k3m_amd.synthetic import synthetic_batch
    cfg = pretrain_config(os.path.join(HERE, "configs", "bert_base_6layer_6conect.json"))
    B = args.batch
    tr = Trainer(cfg, dev, lr=1e-4, warmup_steps=max(1, (args.steps + args.warmup) // 10),
                 total_steps=10 * (args.steps + args.warmup), seed=1234, init=True, dtype=args.dtype)
    if world > 1:
        ddp = GradAllReducer(tr.engine.fp)
        ddp.broadcast_params(tr.engine.fp)
        tr.ddp = ddp
    batch = synthetic_batch(cfg, B, dev, seed=1234 + rank)
    T, P = batch["input_ids"].shape[1], batch["input_ids_pv"].shape[1]
    probe = GemmProbe(2 * B * T + 2 * B * P, cfg.intermediate_size, cfg.hidden_size)
    probe.install()

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        tr.step(batch)
    barrier()
    probe.active = True
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = tr.step(batch)
    barrier()
    dt = time.perf_counter() - t0
    probe.active = False
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([dt], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t)
    loss = float(out["loss"])
    ms_step = 1000.0 * dt / args.steps
    value = world * B * args.steps / dt
    gemm_ms = probe.mean_ms()
    Mg, Ng, Kg = probe.key
    gemm_flops = 2.0 * Mg * Ng * Kg
    achieved = gemm_flops / (gemm_ms * 1e-3) if gemm_ms else None
    bf = args.dtype == "bf16"
    from k3m_amd import ops as _ops, _lib as _L
    x6 = not bf and _ops.F32_ALGO == _L.F32_SPLIT_BF16X6
    peak = PEAK_BF16_MFMA if bf else (PEAK_F32_X6 if x6 else PEAK_F32_MFMA)
    kname = "gemm_bf16_kernel" if bf else ("gemm_x6_kernel" if x6 else "gemm_f32_kernel")
    res = {
        "metric": "pretrain samples/sec (whole job; bert_base_6layer_6conect, bs=64/GPU)",
        "value": round(value, 3), "unit": "samples/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": args.dtype, "data": "synthetic (SURVEY §8(d): random token ids, 36x2048 region feats, 10 PV triples)",
        "config": {"workload": "config %d: bert_base_6layer_6conect %s bs=%d/GPU T=36 P=128 R=37 10 triples" % (
                       3 if bf else 2, "bf16 encoder (fp32 master weights, heads, AdamW)" if bf else "fp32", B),
                   "model": "bert_base_6layer_6conect", "global_batch": B * world, "seq_len": T,
                   "parallelism": "dp%d" % world},
        "per_gpu_samples_s": round(value / world, 3),
        "loss": round(loss, 4),
        "step_mfma_frac_vs_ref_flops": round(B * REF_FLOPS_PER_SAMPLE / (ms_step * 1e-3) / peak, 4),
        "roofline": {"bound": "mfma", "kernel": "%s text-layer FFN1 %dx%dx%d" % (kname, Mg, Ng, Kg),
                     "achieved": round(achieved / 1e12, 2) if achieved else None,
                     "peak": peak / 1e12, "unit": "TFLOP/s",
                     "frac": round(achieved / peak, 4) if achieved else None,
                     "avg_launch_ms": round(gemm_ms, 4) if gemm_ms else None,
                     "launches": len(probe.events),
                     "peak_basis": ("bf16 dense MFMA" if bf else "fp32 via 6 bf16 MFMA partial products = bf16 dense peak / 6"
                                    if x6 else "f32 MFMA"),
                     "traffic": pmc_traffic(probe.key, kname),
                     "traffic_unit": "bytes/launch (rocprofv3 PMC, profiles/r1_gemm_ffn1_pmc.json)"},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            res["cpu_baseline"] = cpu_baseline(cfg, args.cpu_batch, args.cpu_steps)
        except Exception as e:  # baseline only; never masks the GPU result
            res["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
