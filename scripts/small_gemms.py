"""fp32 GEMMs of one training step that fall below the persistent-walk threshold (fewer than K3M_X6_P_MIN 256x128
tiles): shape, layout, epilogue, split-K — to see what runs on the 128x128 / 64x64 x6 tiles.
usage: python scripts/small_gemms.py [--config 3]"""
import argparse
import collections
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    args = ap.parse_args()
    import torch
    import bench
    from k3m_amd import ops, _lib as L
    from k3m_amd.config import pretrain_config
    from k3m_amd.trainer import Trainer
    from k3m_amd.synthetic import synthetic_batch
    from k3m_amd.engine import label_counts
    shape = dict(bench.CONFIGS[args.config])
    dev = torch.device("cuda", 0)
    cfg = pretrain_config(os.path.join(HERE, "configs", "bert_base_6layer_6conect.json"))
    tr = Trainer(cfg, dev, lr=1e-4, warmup_steps=2, total_steps=100, seed=1234, init=True, dtype=shape["dtype"])
    batch = synthetic_batch(cfg, shape["B"], dev, seed=1234, T=shape["T"], P=shape["P"], n_boxes=shape["nbox"],
                            n_triples=shape["n_triples"], npv=shape["npv"])
    batch["_label_counts"] = label_counts(batch)
    tr.step(batch)
    torch.cuda.synchronize()
    seen = collections.Counter()
    orig = L.call

    def call(name, *a):
        if name == "k3m_gemm":
            g = a[0]._obj
            nb = ((g.m + 255) // 256) * ((g.n + 127) // 128) * max(1, g.splitk)
            if g.dtype == L.F32 and nb < 100:
                seen[(g.m, g.n, g.k, g.a_trans, g.b_trans, g.epilogue & 0xff, g.splitk)] += 1
        return orig(name, *a)

    L.call = call
    ops.call = call
    tr.step(batch)
    torch.cuda.synchronize()
    for k, v in sorted(seen.items(), key=lambda kv: -kv[0][0] * kv[0][1] * kv[0][2]):
        print("m=%6d n=%6d k=%6d at=%d bt=%d epi=%d splitk=%d  x%d" % (k + (v,)))


if __name__ == "__main__":
    main()
