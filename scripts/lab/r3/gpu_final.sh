#!/bin/bash
# Final evidence of a build: bench lines for configs 2 (with the CPU baseline), 3, 4, 5 and rocprofv3 kernel
# statistics + traces of configs 2 and 3.  Output under gpurun_out/final/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/final/bench2.json 2> gpurun_out/final/bench2.err || exit 1
echo "config 2 ok"
timeout -k 10 300 python bench.py --config 3 --no-cpu-baseline > gpurun_out/final/bench3.json 2>/dev/null || exit 1
timeout -k 10 400 python bench.py --config 4 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/final/bench4.json 2>/dev/null || exit 1
timeout -k 10 400 python bench.py --config 5 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/final/bench5.json 2>/dev/null || exit 1
echo "configs 3-5 ok"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof2 -o run -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/final/prof2.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof3 -o run -- python bench.py --config 3 --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/final/prof3.log 2>&1 || exit 1
echo "profiles ok"
for f in 2 3 4 5; do tail -n 1 gpurun_out/final/bench$f.json | cut -c1-200; done
