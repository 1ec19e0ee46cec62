"""RCCL (torch "nccl" backend on ROCm) on the GPU box at world size 1: the data-parallel path that replaces
apex DDP (train_concap_struc.py:157-161 process group, :303-308 DDP wrap) executed through RCCL itself,
not gloo.

* scripts/ddp_engine_check.py --world 1 --backend nccl: GradAllReducer's buckets fire in the engine's
  grad-ready order on the comm stream, the RCCL-reduced gradient equals the local gradient (fp32 buckets
  exactly to rounding; bf16 buckets: cast -> all-reduce -> cast back on the comm stream, 2e-2 of scale),
  and the Trainer step leaves finite, identical parameters;
* bench.py --ddp --backend nccl at one rank: the bench's multi-rank line (world_size_seen,
  allreduce_exposed_ms / busy, bucket count, comm dtype, bytes per rank) from a real RCCL run.
Both run in fresh child processes that initialise RCCL before any GPU call of this process."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def _gpu():
    import torch
    if torch.cuda.device_count() < 1:
        pytest.skip("no GPU")


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_rccl_world1_engine_allreduce(dtype):
    _gpu()
    r = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "ddp_engine_check.py"), "--world", "1",
                        "--backend", "nccl", "--dtype", dtype], capture_output=True, text=True, timeout=280,
                       env=_env(), cwd=REPO)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert line, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    res = json.loads(line[-1])
    print(res)
    assert res["backend"] == "nccl" and res["world_seen"] == 1 and res["dtype"] == dtype
    assert res["order_ok"], res
    assert res["max_rel_err_vs_sum_of_local"] < res["tolerance"], res
    assert r.returncode == 0 and res["ok"], res


@pytest.mark.parametrize("config", [2, 3])
def test_rccl_world1_bench_line(config):
    """config 2: fp32 buckets; config 3: bf16 encoder with bf16 buckets."""
    _gpu()
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--ddp", "--backend", "nccl", "--config",
                        str(config), "--batch", "8", "--steps", "3", "--warmup", "2", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=280, env=_env(), cwd=REPO)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and line, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    res = json.loads(line[-1])
    print({k: res.get(k) for k in ("value", "ms_per_step", "backend", "world_size_seen", "allreduce_exposed_ms",
                                   "allreduce_busy_ms", "allreduce_buckets_per_step", "allreduce_dtype",
                                   "grad_bytes_per_rank")})
    assert res["backend"] == "nccl" and res["world_size_seen"] == 1 and res["n_gpus"] == 1
    assert res["allreduce_dtype"] == ("bf16" if config == 3 else "fp32")
    assert res["allreduce_buckets_per_step"] > 20
    assert res["allreduce_exposed_ms"] >= 0.0 and res["allreduce_busy_ms"] > 0.0
    assert res["grad_bytes_per_rank"] > (0.8e9 if config == 3 else 1.6e9)
    assert res["value"] > 0 and res["loss"] == res["loss"]
