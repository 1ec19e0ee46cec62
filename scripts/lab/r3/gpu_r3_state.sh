#!/bin/bash
# Round-3 state: bench lines (fp32 config 2, bf16 configs 3-5) with host issue time, kernel roofline table.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -n 1 "gpurun_out/$name.log" | cut -c1-400; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
run b2 300 python bench.py --no-cpu-baseline --steps 10 --warmup 4
run b3 300 python bench.py --config 3 --no-cpu-baseline --steps 10 --warmup 4
run b4 400 python bench.py --config 4 --no-cpu-baseline --steps 5 --warmup 2
run b5 400 python bench.py --config 5 --no-cpu-baseline --steps 5 --warmup 2
run kr 400 python scripts/kernel_roofline.py r3_kernel_roofline
