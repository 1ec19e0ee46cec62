#!/bin/bash
# final round-6 records: GPU suite + smoke, bench lines of configs 2 (with the CPU baseline and oracle parity), 3, 4, 5
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r6final
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.txt 2>&1
rc=$?
tail -2 $out/gpu_tests.txt
[ $rc -eq 0 ] || { grep -E "Error|FAILED" $out/gpu_tests.txt | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.txt 2>&1 || { tail -20 $out/smoke.txt; exit 1; }
tail -1 $out/smoke.txt
timeout -k 10 600 python bench.py > $out/bench_cfg2.json 2> $out/bench_cfg2.err || { tail -20 $out/bench_cfg2.err; exit 1; }
for c in 3 4 5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline > $out/bench_cfg$c.json 2> $out/bench_cfg$c.err || { tail -20 $out/bench_cfg$c.err; exit 1; }
done
for c in 2 3 4 5; do
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print($c, d['value'], d['ms_per_step'], d.get('roofline', {}).get('frac'), d.get('parity', {}).get('max_rel') if isinstance(d.get('parity'), dict) else '')" $out/bench_cfg$c.json
done
