"""Every GEMM launch of one training step (bench.py's workload, eager issue): shape, layout, epilogue, split-K,
grouped or not, HIP-event time and TF/s, aggregated per call signature and sorted by total time.
usage: python scripts/gemm_calls.py [--config 2] [--top 40]"""
import argparse
import collections
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--top", type=int, default=40)
    args = ap.parse_args()
    import torch
    import bench
    from k3m_amd import _lib as L, ops
    from k3m_amd.config import pretrain_config
    from k3m_amd.trainer import Trainer
    from k3m_amd.synthetic import synthetic_batch
    from k3m_amd.engine import label_counts
    shape = dict(bench.CONFIGS[args.config])
    dev = torch.device("cuda", 0)
    cfg = pretrain_config(os.path.join(HERE, "configs", "bert_base_6layer_6conect.json"))
    tr = Trainer(cfg, dev, lr=1e-4, warmup_steps=2, total_steps=100, seed=1234, dtype=shape["dtype"])
    tr.graph = False
    batch = synthetic_batch(cfg, shape["B"], dev, seed=1234, T=shape["T"], P=shape["P"], n_boxes=shape["nbox"],
                            n_triples=shape["n_triples"], npv=shape["npv"])
    batch["_label_counts"] = label_counts(batch)
    rec = []
    active = [False]
    orig = L.call

    def sig(g):
        return "%s%s m=%d n=%d k=%d epi=%d s=%d" % ("t" if g.a_trans else "n", "t" if g.b_trans else "n", g.m, g.n, g.k,
                                                    g.epilogue & 0xff, g.splitk)

    def wrapped(name, *a):
        if not active[0] or name not in ("k3m_gemm", "k3m_gemm_grouped"):
            return orig(name, *a)
        if name == "k3m_gemm":
            gs = [a[0]._obj]
        else:
            arr = L.C.cast(a[0], L.C.POINTER(L.K3mGemm))
            gs = [arr[i] for i in range(a[1])]
        key = ("group[%d] " % len(gs) if name == "k3m_gemm_grouped" else "") + " + ".join(sig(g) for g in gs)
        flops = sum(2.0 * g.m * g.n * g.k for g in gs)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        r = orig(name, *a)
        e.record()
        rec.append((key, flops, s, e))
        return r
    L.call = wrapped
    ops.call = wrapped
    for _ in range(3):
        tr.step(batch)
    torch.cuda.synchronize()
    active[0] = True
    tr.step(batch)
    torch.cuda.synchronize()
    active[0] = False
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for key, flops, s, e in rec:
        a = agg[key]
        a[0] += 1
        a[1] += s.elapsed_time(e)
        a[2] += flops
    tot = sum(v[1] for v in agg.values())
    print("GEMM launches in one step: %d, %.2f ms (HIP events; the step's other kernels excluded)" % (len(rec), tot))
    for key, (n, ms, fl) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:args.top]:
        print("%3d x %8.3f ms  %6.1f TF/s  %4.1f%%  %s" % (n, ms / n, fl / (ms * 1e-3) / 1e12, 100 * ms / tot, key[:220]))


if __name__ == "__main__":
    main()
