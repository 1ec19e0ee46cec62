#!/bin/bash
# HEAD (x6 ping-pong default 63): GPU suite, smoke, default bench line, config-2 profile, configs 3 and 5 lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r5e_gpu_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/r5e_gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5e_smoke.txt 2>&1 || { tail -20 gpurun_out/r5e_smoke.txt; exit 1; }
tail -1 gpurun_out/r5e_smoke.txt
timeout -k 10 600 python bench.py > gpurun_out/r5e_bench_cfg2.json 2> gpurun_out/r5e_bench_cfg2.err || exit 1
tail -1 gpurun_out/r5e_bench_cfg2.json | cut -c1-400
bash scripts/prof_cfg.sh 2 r5e_cfg2 2 || exit 1
head -3 gpurun_out/prof_r5e_cfg2/step_split.txt; head -2 gpurun_out/prof_r5e_cfg2/gemm_calls.txt
timeout -k 10 600 python bench.py --config 3 --steps 10 --warmup 4 --no-cpu-baseline > gpurun_out/r5e_bench_cfg3.json 2>/dev/null || exit 1
tail -1 gpurun_out/r5e_bench_cfg3.json | cut -c1-200
timeout -k 10 900 python bench.py --config 5 --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/r5e_bench_cfg5.json 2>/dev/null || exit 1
tail -1 gpurun_out/r5e_bench_cfg5.json | cut -c1-200
