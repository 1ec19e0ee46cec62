#!/bin/bash
# Same-box A/B of two builds of libk3m_hip.so: interleaved bench.py runs, one line each.
# usage: scripts/ab_lib.sh A.so B.so ROUNDS [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
a=$1; b=$2; rounds=$3; shift 3
for r in $(seq 1 "$rounds"); do
  for lib in "$a" "$b"; do
    out=$(K3M_LIB="$lib" timeout -k 10 300 python bench.py --no-cpu-baseline "$@" 2>/dev/null | tail -n 1)
    rc=$?
    if [ $rc -ne 0 ]; then echo "$lib rc=$rc"; exit $rc; fi
    echo "$(basename "$lib") $(echo "$out" | python -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["coattn"]["frac"])')"
  done
done
