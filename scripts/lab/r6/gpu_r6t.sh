#!/bin/bash
# config-2 runtime knobs on the current build, same box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
bash scripts/ab_env_bench.sh 2 K3M_BRANCH_STREAMS "1 2 4" 2 r6t || exit 1
bash scripts/ab_env_bench.sh 2 K3M_OPT_OVERLAP "1 0" 2 r6t || exit 1
for r in 1 2; do
  for g in auto on; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --graph $g > gpurun_out/r6t/graph_${g}_$r.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print('graph=$g round $r', d['value'], d['ms_per_step'], d['graph'])" gpurun_out/r6t/graph_${g}_$r.json
  done
done
