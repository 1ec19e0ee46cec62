#!/bin/bash
# same-box interleaved A/B of one environment knob on a bench config
# usage: scripts/ab_env_bench.sh CONFIG VAR "VALUES" ROUNDS TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cfg=$1; var=$2; vals=$3; rounds=${4:-2}; tag=${5:-ab}
mkdir -p gpurun_out/$tag
for r in $(seq 1 $rounds); do
  for v in $vals; do
    out=gpurun_out/$tag/cfg${cfg}_${var}_${v}_r${r}.json
    env "$var=$v" timeout -k 10 300 python bench.py --config "$cfg" --no-cpu-baseline > "$out" 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('$var=$v round $r', d['value'], d['ms_per_step'])" "$out" || exit 1
  done
done
