#!/bin/bash
# PMC record of the largest GEMM class at HEAD: the FFN2 -> dGELU input gradient (ping-pong walk)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/pmc_gemm.sh r5edg "dgrad ffn2->dgelu" fp32 || exit 1
# algorithmic bytes: A 20992x768, B 768x3072, aux 20992x3072 read, C 20992x3072 written (fp32)
python scripts/pmc_table.py r5edg "gemm_x6_persist_kernel<256, 256, 2, 4, 16, true, false, 3, true, 1>" 99052683264 589824000 20992,3072,768 > gpurun_out/r5e_pmc_x6_dgelu_pp.json || exit 1
python - <<'PY'
import json
d = json.load(open("gpurun_out/r5e_pmc_x6_dgelu_pp.json"))
print({k: (round(v, 4) if isinstance(v, float) else v) for k, v in d.items() if k not in ("counters_mean_per_dispatch", "dispatches", "kernel_names")})
PY
