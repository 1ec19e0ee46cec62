#!/bin/bash
# same-box interleaved A/B of two library builds (K3M_LIB) on a bench config
# usage: scripts/ab_lib_bench.sh CONFIG PREV_LIB ROUNDS TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cfg=$1; prev=$2; rounds=${3:-2}; tag=${4:-ablib}
mkdir -p gpurun_out/$tag
for r in $(seq 1 $rounds); do
  for v in new prev; do
    out=gpurun_out/$tag/cfg${cfg}_${v}_r${r}.json
    if [ $v = prev ]; then lib="$prev"; else lib=k3m_amd/libk3m_hip.so; fi
    K3M_LIB="$lib" timeout -k 10 300 python bench.py --config "$cfg" --no-cpu-baseline > "$out" 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('$v round $r', d['value'], d['ms_per_step'])" "$out" || exit 1
  done
done
