"""cProfile of the host side of Trainer.step (bench.py's workload): where the Python engine spends the
time it takes to issue one step.  usage: python scripts/host_profile.py [--config 3] [--steps 5]"""
import argparse
import cProfile
import os
import pstats
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--top", type=int, default=45)
    args = ap.parse_args()
    import torch
    import bench
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
    for _ in range(3):
        tr.step(batch)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(args.steps):
        tr.step(batch)
        torch.cuda.synchronize()   # host time of each step alone, not queued behind the GPU
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(args.top)
    st.sort_stats("cumulative").print_stats(args.top)


if __name__ == "__main__":
    main()
