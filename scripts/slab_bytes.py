"""Bytes the deferred slab reductions move per step (slab reads + output read/write), to price slab_batch_kernel
against its HBM roofline.  usage: python scripts/slab_bytes.py [--config 2]"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    args = ap.parse_args()
    import torch
    import bench
    from k3m_amd import ops
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
    stats = {"flushes": 0, "jobs": 0, "slab_bytes": 0, "out_bytes": 0, "by_nslab": {}}
    orig = ops._Deferred.flush

    def flush(self):
        if self.jobs:
            stats["flushes"] += 1
            for _, _, ns, cols, acc in self.jobs:
                stats["jobs"] += 1
                stats["slab_bytes"] += 4 * ns * cols
                stats["out_bytes"] += 4 * cols * (2 if acc else 1)
                key = "nslab<=64" if ns <= 64 else "nslab>64"
                stats["by_nslab"][key] = stats["by_nslab"].get(key, 0) + 4 * ns * cols
        return orig(self)

    ops._Deferred.flush = flush
    tr.step(batch)
    torch.cuda.synchronize()
    print(stats)
    print("GB per step: slabs %.3f, outputs %.3f" % (stats["slab_bytes"] / 1e9, stats["out_bytes"] / 1e9))


if __name__ == "__main__":
    main()
