#!/bin/bash
# Round-3 GPU check: the GPU tests most affected by a change, then the A/B and config bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/gputests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/ab_env.sh K3M_DEFER_REDUCE "0 1" 2 --config 3 --steps 10 --warmup 3 || exit $?
bash scripts/ab_env.sh K3M_DEFER_REDUCE "0 1" 2 --steps 10 --warmup 3 || exit $?
for c in 4 5; do
  timeout -k 10 400 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench$c.log 2>&1 || exit $?
  grep '^{' gpurun_out/bench$c.log | cut -c1-400
done
