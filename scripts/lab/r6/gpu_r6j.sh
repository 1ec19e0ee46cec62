#!/bin/bash
# bench lines of configs 5, 3, 2 (no CPU baseline) after the pair-draw attention dropout
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r6j
for c in 5 3 2; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > gpurun_out/r6j/bench_cfg$c.json 2> gpurun_out/r6j/bench_cfg$c.err || { tail -20 gpurun_out/r6j/bench_cfg$c.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/r6j/bench_cfg$c.json')); print($c, d['value'], d['ms_per_step'])"
done
