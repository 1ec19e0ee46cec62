#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/pmc_attn_long.sh r6fl || exit 1
python scripts/pmc_table.py r6fl "flash_long_bwd2_kernel<64>" 201326592000 > gpurun_out/r6_pmc_flash_long_bwd2_pair.json || exit 1
python scripts/pmc_table.py r6fl "flash_long_fwd2_kernel<64>" 80530636800 > gpurun_out/r6_pmc_flash_long_fwd2_pair.json || exit 1
for f in gpurun_out/r6_pmc_flash_long_*_pair.json; do
python -c "
import json,sys; d=json.load(open('$f'))
m=d['counters_mean_per_dispatch']
print('$f', {k: (round(v, 4) if isinstance(v, float) else v) for k, v in d.items() if k not in ('counters_mean_per_dispatch', 'dispatches', 'kernel_names')})
print({k: round(v) for k, v in m.items()})"
done
