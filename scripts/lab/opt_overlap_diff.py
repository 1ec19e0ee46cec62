"""Debug: which parameter tensors differ between the overlapped per-block AdamW and the single sweep."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    from k3m_amd.trainer import Trainer
    from k3m_amd.synthetic import synthetic_batch, synthetic_noise
    from test_gpu_trainer import _no_dropout_cfg, _fixed_negs
    dev = torch.device("cuda")
    cfg = _no_dropout_cfg()
    B = 2
    batch = synthetic_batch(cfg, B, dev, seed=41)
    noise = {k: v.to(dev) for k, v in synthetic_noise(cfg, B, seed=51).items()}
    ent, val = _fixed_negs(B, 20, 10)
    res = []
    for mode in ("sweep", "sweep2", "overlap", "overlap_sync"):
        tr = Trainer(cfg, dev, lr=1e-3, warmup_steps=1, total_steps=10, seed=5, nan_check=False)
        tr.overlap = not mode.startswith("sweep")
        if mode == "overlap_sync":
            orig = tr._overlap_block

            def blk(b, orig=orig):
                torch.cuda.synchronize()
                orig(b)
                torch.cuda.synchronize()
            tr._overlap_block = blk
        tr.step(batch, noise=noise, ent_neg=ent, val_neg=val)
        torch.cuda.synchronize()
        res.append((mode, tr.m.clone(), tr.engine.fp.grad.clone(), tr))
    fp = res[0][3].engine.fp
    print("sweep grad nonzero after step:", int((res[0][2] != 0).sum()), flush=True)
    for mode, p, g, _ in res[1:]:
        print(mode, "grad nonzero after step:", int((g != 0).sum()), flush=True)
        bad = []
        for name, shape in fp.spec:
            o = fp.offsets[name]
            n = 1
            for s_ in shape:
                n *= s_
            a, b = res[0][1][o:o + n], p[o:o + n]
            if not torch.equal(a, b):
                bad.append((float((a - b).abs().max()), name))
        bad.sort(reverse=True)
        print(mode, "differing exp_avg tensors after step 1:", len(bad), bad[:15], flush=True)


if __name__ == "__main__":
    main()
