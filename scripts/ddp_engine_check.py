"""Two-rank data-parallel check of the real engine: each rank runs the K3M step
on its own half-batch; the gradient all-reduce (k3m_amd.ddp.GradAllReducer, the replacement of
apex DDP, train_concap_struc.py:303-308) must

* fire its buckets in the engine's real grad-ready order: heads/fusion/structure first, then every
  encoder block in reverse schedule order as its backward finishes, embeddings last;
* produce, on every rank, exactly the sum of the ranks' single-process gradients (checked on
  tensors of every block kind and on whole-buffer checksums);
* leave identical parameters on all ranks after Trainer.step (all-reduce + AdamW with 1/world).

Dropout is off and the gumbel noise / LPM negatives are explicit, so a rank's second backward
repeats its first.  Both ranks may share one GPU (``--backend gloo``); with one GPU per rank use nccl
(RCCL).  The parent never touches the GPU (the ranks are child processes).  Prints one JSON line.

    python scripts/ddp_engine_check.py [--world 2] [--backend gloo] [--batch 2]
"""
import argparse
import json
import os
import socket
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)

NAMES = ["cls.predictions.transform.dense.weight", "struc_w1.weight", "score_self_t.weight",
         "encoder.c_layer.5.biattention.query1.weight", "encoder.c_layer_pv_t.0.t_output.dense.bias",
         "encoder.v_layer.3.output.dense.weight", "encoder.layer.11.intermediate.dense.weight",
         "encoder.layer.0.attention.self.query.weight", "embeddings.word_embeddings.weight",
         "v_embeddings.image_embeddings.weight"]


def _worker(rank, world, port, backend, batch_size, out, dtype="fp32"):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    ndev = torch.cuda.device_count()
    torch.cuda.set_device(rank % ndev)
    dev = torch.device("cuda", rank % ndev)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
    from k3m_amd.config import pretrain_config
    from k3m_amd.ddp import GradAllReducer
    from k3m_amd.synthetic import synthetic_batch, synthetic_noise
    from k3m_amd.trainer import Trainer
    cfg = pretrain_config(os.path.join(REPO, "configs", "bert_base_6layer_6conect.json"))
    cfg.hidden_dropout_prob = cfg.attention_probs_dropout_prob = 0.0
    cfg.v_hidden_dropout_prob = cfg.v_attention_probs_dropout_prob = 0.0
    B = batch_size
    tr = Trainer(cfg, dev, lr=1e-3, warmup_steps=0, total_steps=10, seed=5, dtype=dtype)
    eng = tr.engine
    batch = synthetic_batch(cfg, B, dev, seed=100 + rank)
    noise = {k: v.to(dev) for k, v in synthetic_noise(cfg, B, seed=200 + rank).items()}
    ent = torch.full((B, 20, 2), -1, dtype=torch.int64)
    val = torch.full((B, 20, 2), -1, dtype=torch.int64)
    for i in range(B):
        for j in range(10):
            ent[i, j, 0] = (i + 1) % B if B > 1 else -1
            val[i, j, 0], val[i, j, 1] = (j + 1) % 10, (j + 2) % 10

    def fwd_bwd(hook=None):
        out, ctx = eng.forward(batch, train=True, noise=noise, ent_neg=ent, val_neg=val)
        eng.backward(ctx, grad_ready=hook)
        return out

    eng.fp.grad.zero_()
    fwd_bwd()
    torch.cuda.synchronize()
    local = {n: eng.fp.g[n].detach().cpu().clone() for n in NAMES}
    local_sum = float(eng.fp.grad.double().sum())
    local_abs = float(eng.fp.grad.double().abs().sum())
    eng.fp.grad.zero_()

    ddp = GradAllReducer(eng.fp, comm_dtype=torch.bfloat16 if dtype == "bf16" else None)
    order = []
    orig = ddp._launch

    def rec(blk):
        if blk not in ddp.done and blk in ddp.blocks:
            order.append(list(blk))
        return orig(blk)
    ddp._launch = rec
    ddp.begin(eng)
    fwd_bwd(ddp.grad_ready)
    ddp.finish()
    torch.cuda.synchronize()
    reduced = {n: eng.fp.g[n].detach().cpu().clone() for n in NAMES}
    reduced_sum = float(eng.fp.grad.double().sum())
    eng.fp.grad.zero_()

    ddp._launch = orig
    tr.ddp = ddp
    tr.step(batch, noise=noise, ent_neg=ent, val_neg=val)
    torch.cuda.synchronize()
    psum = float(eng.fp.data.double().sum())
    pabs = float(eng.fp.data.double().abs().sum())
    torch.save({"local": local, "reduced": reduced, "local_sum": local_sum, "local_abs": local_abs, "reduced_sum": reduced_sum,
                "order": order, "schedule": [list(x) for x in eng.schedule], "psum": psum, "pabs": pabs,
                "world_seen": dist.get_world_size()}, os.path.join(out, "r%d.pt" % rank))
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--backend", default="gloo")
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"],
                    help="bf16: bf16 encoder and bf16 gradient buckets (reduced-gradient tolerance 1e-2)")
    a = ap.parse_args()
    import torch
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = tempfile.mkdtemp(prefix="k3m_ddp_")
    mp.spawn(_worker, args=(a.world, port, a.backend, a.batch, out, a.dtype), nprocs=a.world, join=True)
    R = [torch.load(os.path.join(out, "r%d.pt" % r), weights_only=True) for r in range(a.world)]
    sched = R[0]["schedule"]
    expected = [["head", 0]] + [[k, i] for k, i in reversed(sched)] + [["emb", 0]]
    res = {"world": a.world, "backend": a.backend, "dtype": a.dtype, "world_seen": R[0]["world_seen"],
           "order_ok": all(r["order"] == expected for r in R), "order_rank0": R[0]["order"][:6] + ["..."]}
    worst = 0.0
    for n in NAMES:
        want = sum(r["local"][n].double() for r in R)
        scale = float(want.abs().max()) + 1e-12
        for r in R:
            worst = max(worst, float((r["reduced"][n].double() - want).abs().max()) / scale)
    res["max_rel_err_vs_sum_of_local"] = worst
    res["ranks_bitwise_equal"] = all(torch.equal(R[0]["reduced"][n], r["reduced"][n]) for r in R for n in NAMES)
    # whole-buffer checksum: sum(reduced) == sum_r sum(local_r), relative to sum_r sum|local_r| (the
    # signed sum cancels, so it is not its own scale)
    want_sum = sum(r["local_sum"] for r in R)
    abs_scale = sum(r["local_abs"] for r in R) + 1e-12
    res["checksum_rel_err"] = max(abs(r["reduced_sum"] - want_sum) / abs_scale for r in R)
    res["params_equal_after_step"] = all(r["psum"] == R[0]["psum"] and r["pabs"] == R[0]["pabs"] for r in R)
    # fp32 buckets: the sum is exact to fp32 rounding; bf16 buckets round each rank's gradient and the
    # partial sums to 8 significant bits (2^-8 relative per rounding, a few roundings per element)
    tol, ctol = (1e-5, 1e-6) if a.dtype == "fp32" else (2e-2, 1e-2)
    res["tolerance"] = tol
    res["ok"] = bool(res["order_ok"] and worst < tol and res["ranks_bitwise_equal"] and
                     res["checksum_rel_err"] < ctol and res["params_equal_after_step"] and
                     res["world_seen"] == a.world)
    print(json.dumps(res), flush=True)
    sys.exit(0 if res["ok"] else 1)


if __name__ == "__main__":
    main()
