#!/bin/bash
# Same-box A/B: the round's starting tree (_old/, commit 6819e76, its own build) vs this tree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['coattn']['frac'])" "$1"; }
for r in 1 2 3; do
  (cd _old && timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 4) | summ "start fp32" || exit 1
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 4 | summ "head  fp32" || exit 1
done
for r in 1 2; do
  (cd _old && timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline --steps 10 --warmup 4) | summ "start bf16" || exit 1
  timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline --steps 10 --warmup 4 | summ "head  bf16" || exit 1
done
