"""Data-parallel step on the real engine, two ranks over gloo sharing GPU 0 (the driver's 8-GPU
RCCL run uses the same code with backend nccl): bucket order = real grad-ready order, reduced
gradient = sum of the ranks' single-process gradients, identical parameters after the step.
The ranks run in child processes (scripts/ddp_engine_check.py) so this process's GPU state is not
inherited."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_two_rank_engine_allreduce(dtype):
    """fp32: fp32 buckets; bf16: the bf16 encoder with bf16 gradient buckets (cast on the comm stream)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "ddp_engine_check.py"), "--world", "2",
                        "--backend", "gloo", "--dtype", dtype], capture_output=True, text=True, timeout=280, env=env,
                       cwd=REPO)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert line, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    res = json.loads(line[-1])
    print(res)
    assert res["order_ok"], res
    assert res["ranks_bitwise_equal"] and res["max_rel_err_vs_sum_of_local"] < res["tolerance"], res
    assert res["dtype"] == dtype
    assert res["params_equal_after_step"] and res["world_seen"] == 2, res
    assert r.returncode == 0 and res["ok"], res
