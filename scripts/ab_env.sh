#!/bin/bash
# A/B a library env knob on one box: interleaved bench runs, one JSON line each.
# usage: scripts/ab_env.sh VAR "v1 v2 ..." ROUNDS [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
var=$1; vals=$2; rounds=$3; shift 3
for r in $(seq 1 "$rounds"); do
  for v in $vals; do
    out=$(env "$var=$v" timeout -k 10 300 python bench.py --no-cpu-baseline "$@" 2>/dev/null | tail -n 1)
    rc=$?
    if [ $rc -ne 0 ]; then echo "$var=$v rc=$rc"; exit $rc; fi
    echo "$var=$v $(echo "$out" | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"])')"
  done
done
