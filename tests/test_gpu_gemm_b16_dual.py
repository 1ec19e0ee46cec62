"""The two-workgroups-per-CU bf16 GEMM (gemm_b16_tile.h gemm_dual_kernel, K3M_B16_DUAL=1) computes every
element with the same bf16 products accumulated in the same k order as the 8-wave walk, so its C (and the
GELU pre-activation) must be BIT-IDENTICAL on every layout, epilogue, split-K and grouped launch
(scripts/b16_dump.py in child processes with K3M_B16_DUAL = 0 / 1 / 2, the knob being read at library load)."""
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_dual_kernel_bit_identical(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    outs = {}
    for dual in ("0", "1", "2"):
        env = dict(os.environ, K3M_B16_DUAL=dual)
        out = str(tmp_path / ("c%s.pt" % dual))
        r = subprocess.run([sys.executable, os.path.join(REPO, "scripts", "b16_dump.py"), out], env=env, cwd=REPO,
                           capture_output=True, text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-3000:]
        outs[dual] = torch.load(out, weights_only=True)
    for d in ("1", "2"):
        assert sorted(outs["0"]) == sorted(outs[d])
        for k in outs["0"]:
            a, b = outs["0"][k], outs[d][k]
            assert torch.isfinite(a.float()).all(), k
            assert torch.equal(a, b), (d, k, float((a.float() - b.float()).abs().max()))
