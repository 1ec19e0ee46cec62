#!/bin/bash
# tile thresholds for the mid-size fp32 GEMMs (image embedding 2,368 x 1,024 x 2,048, the 1,280- and 1,552-row
# head GEMMs): persistent 256x128 walk from K3M_X6_P_MIN tiles, 128x128 tiles from K3M_X6_T128_MIN, else 64x64
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2; do
  for cfg in "100 200" "30 200" "100 50" "30 50"; do
    set -- $cfg
    out=$(K3M_X6_P_MIN=$1 K3M_X6_T128_MIN=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --config 2 --steps 12 2>/dev/null | tail -n 1)
    echo "P_MIN=$1 T128_MIN=$2 $(echo "$out" | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"])')"
  done
done
