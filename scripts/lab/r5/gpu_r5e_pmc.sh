#!/bin/bash
# HEAD PMC records: the FFN1 forward (ping-pong) and the ffn1 weight gradient (LDS-DMA-staged ping-pong)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/pmc_gemm.sh r5effn1 "fwd ffn1 gelu" fp32 || exit 1
python scripts/pmc_table.py r5effn1 "gemm_x6_persist_kernel<256, 256, 4, 2, 16, true, true, 2, true, 1>" 99052683264 589824000 20992,3072,768 > gpurun_out/r5e_pmc_x6_ffn1_pp.json || exit 1
bash scripts/pmc_gemm.sh r5ewg "wgrad ffn1" fp32 || exit 1
python scripts/pmc_table.py r5ewg "gemm_x6_persist_kernel<256, 256, 2, 4, 16, false, false, 0, false, 2>" 99052683264 > gpurun_out/r5e_pmc_wgrad_ppd.json || exit 1
python - <<'PY'
import json
for f in ["gpurun_out/r5e_pmc_x6_ffn1_pp.json", "gpurun_out/r5e_pmc_wgrad_ppd.json"]:
    d = json.load(open(f))
    print(f, {k: (round(v, 4) if isinstance(v, float) else v) for k, v in d.items() if k not in ("counters_mean_per_dispatch", "dispatches", "kernel_names")})
PY
