#!/bin/bash
# rocprofv3 kernel trace + stats of bench.py for one config, then the per-call GEMM table and the step split.
# usage: scripts/prof_cfg.sh CONFIG TAG [steps]      (outputs under gpurun_out/prof_TAG)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
cfg=$1; tag=$2; steps=${3:-2}
out=gpurun_out/prof_$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run -- python bench.py --config "$cfg" --steps "$steps" --warmup 1 --no-cpu-baseline > "$out/bench.log" 2>&1 || exit $?
tr=$(find "$out" -name "run_kernel_trace.csv" | head -1)
st=$(find "$out" -name "run_kernel_stats.csv" | head -1)
python scripts/step_time_split.py "$tr" "$steps" 40 30 > "$out/step_split.txt" 2>&1
python scripts/step_gaps.py "$tr" "$steps" 5 30 > "$out/step_gaps.txt" 2>&1
cp "$st" "$out/kernel_stats.csv"
rm -f "$tr"
timeout -k 10 400 python scripts/gemm_calls.py --config "$cfg" --top 60 > "$out/gemm_calls.txt" 2>&1
