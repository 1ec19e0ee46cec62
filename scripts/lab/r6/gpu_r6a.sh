#!/bin/bash
# round 6, first GPU pass: new fixtures and tests, the default bench line (roofline = weight-gradient walk, parity
# field), the gate flip-rate record and the HEAD PMC record of the dominant kernel's FFN1 weight-gradient shape
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python -u tests/golden/make_flash_long_golden.py > gpurun_out/r6a_golden.log 2>&1 || { tail -30 gpurun_out/r6a_golden.log; exit 1; }
cp tests/golden/flash_long_d96.npz gpurun_out/ || exit 1
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_graph.py tests/test_gpu_fullsize.py "tests/test_gpu_gemm_x6.py::test_small_splitk_epilogues" \
  "tests/test_gpu_gemm_bf16.py::test_flash_long_d96_matches_fixed_seed_golden" \
  "tests/test_gpu_configs.py::test_bf16_matches_fp32_step" > gpurun_out/r6a_tests.log 2>&1 || { tail -40 gpurun_out/r6a_tests.log; exit 1; }
tail -3 gpurun_out/r6a_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/r6a_bench2.json 2> gpurun_out/r6a_bench2.err || { tail -30 gpurun_out/r6a_bench2.err; exit 1; }
tail -c 3000 gpurun_out/r6a_bench2.json
timeout -k 10 300 python -u scripts/gate_flips.py gpurun_out/r6a_gate_flip_rate.json > gpurun_out/r6a_gate_flips.log 2>&1 || { tail -30 gpurun_out/r6a_gate_flips.log; exit 1; }
cat gpurun_out/r6a_gate_flips.log
bash scripts/pmc_gemm.sh r6wg "wgrad ffn1" fp32 || exit 1
python scripts/pmc_table.py r6wg "gemm_x6_persist_kernel<256, 256, 2, 4, 16, false, false, 0, false, 2>" 99052683264 331923456 3072,768,20992 > gpurun_out/r6_pmc_x6_wgrad_ffn1_ppd.json || exit 1
python -c "
import json; d=json.load(open('gpurun_out/r6_pmc_x6_wgrad_ffn1_ppd.json'))
print({k: (round(v, 4) if isinstance(v, float) else v) for k, v in d.items() if k not in ('counters_mean_per_dispatch', 'dispatches', 'kernel_names')})"
