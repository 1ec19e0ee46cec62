#!/bin/bash
# persistent bf16 large-tile walk (K3M_B16_PERSIST=1): bf16 GEMM / config tests with it on, bit-identity of a
# config-3 step's losses and gradients against the one-tile-per-workgroup grid, interleaved config-3 A/B
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
K3M_B16_PERSIST=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gemm_bf16.py > gpurun_out/b16p_tests.txt 2>&1
for v in 0 1; do
  K3M_B16_PERSIST=$v timeout -k 10 200 python - <<PY
import os, sys, torch
sys.path.insert(0, ".")
import bench
from k3m_amd.config import pretrain_config
from k3m_amd.trainer import Trainer
from k3m_amd.synthetic import synthetic_batch
from k3m_amd.engine import label_counts
shape = dict(bench.CONFIGS[3])
dev = torch.device("cuda", 0)
cfg = pretrain_config("configs/bert_base_6layer_6conect.json")
tr = Trainer(cfg, dev, lr=1e-4, warmup_steps=2, total_steps=100, seed=1234, init=True, dtype=shape["dtype"])
b = synthetic_batch(cfg, 16, dev, seed=1234, T=shape["T"], P=shape["P"], n_boxes=shape["nbox"], n_triples=shape["n_triples"], npv=shape["npv"])
b["_label_counts"] = label_counts(b)
tr.step(b)
torch.cuda.synchronize()
torch.save({"p": tr.engine.fp.data[:50_000_000].cpu(), "g0": tr.engine.fp.data[-50_000_000:].cpu()}, "gpurun_out/b16p_%s.pt" % os.environ["K3M_B16_PERSIST"])
PY
done
python -c "
import torch
A=torch.load('gpurun_out/b16p_0.pt',weights_only=True); B=torch.load('gpurun_out/b16p_1.pt',weights_only=True); a=torch.cat([A['p'],A['g0']]); b=torch.cat([B['p'],B['g0']])
print('params after one step bit-identical:', torch.equal(a,b), float((a-b).abs().max()))
" > gpurun_out/b16p_ident.txt 2>&1
rm -f gpurun_out/b16p_0.pt gpurun_out/b16p_1.pt
bash scripts/ab_env.sh K3M_B16_PERSIST "0 1" 3 --config 3 --steps 20 > gpurun_out/b16p_ab.txt 2>&1
