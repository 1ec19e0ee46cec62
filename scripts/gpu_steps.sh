#!/bin/bash
# Run GPU steps in order; stop at the first step that faults / aborts / times out
# (pytest exit 1 = test failures: keep going so later steps still report).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {
  local name=$1 limit=$2; shift 2
  echo "== $name (limit ${limit}s): $*"
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after $name (rc=$rc)"
    exit $rc
  fi
}
for s in "$@"; do
  case $s in
    kern) step kern 400 python -m pytest tests/test_gpu_kernels.py -q ;;
    x6) step x6 400 python -m pytest tests/test_gpu_gemm_x6.py -q ;;
    lab) step lab 300 scripts/lab/gemm_lab 10 ;;
    smoke) step smoke 400 python -c "import __graft_entry__ as g; g.smoke()" ;;
    parity) step parity 900 python -m pytest tests/test_gpu_parity.py -x -q ;;
    gpu) step gputests 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ;;
    bench3) step bench3 600 python bench.py --config 3 --steps 10 --warmup 3 --no-cpu-baseline ;;
    bench4) step bench4 900 python bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline ;;
    bench5) step bench5 900 python bench.py --config 5 --steps 5 --warmup 2 --no-cpu-baseline ;;
    spawn2) step spawn2 600 python bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo --batch 16 ;;
    bench) step bench 600 python bench.py --steps 10 --warmup 3 ;;
    benchq) step bench 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline ;;
    profbf) export TMPDIR=/tmp; step profbf 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profbf -o run -- python bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline ;;
    profbf10) export TMPDIR=/tmp; step profbf10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profbf10 -o run -- python bench.py --config 3 --steps 10 --warmup 2 --no-cpu-baseline ;;
    tbig) step tbig 600 python -u -m pytest tests/test_gpu_gemm_b16_big.py tests/test_gpu_gemm_bf16.py -v --timeout 300 --timeout-method thread ;;
    ddpeng) step ddpeng 400 python -u -m pytest tests/test_gpu_ddp_engine.py -v -s --timeout 300 --timeout-method thread ;;
    ttrain) step ttrain 900 python -u -m pytest tests/test_gpu_trainer.py -v --timeout 300 --timeout-method thread ;;
    prof) export TMPDIR=/tmp; step prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
    gemm) step gemm 300 python scripts/gemm_bench.py all 10 both ;;
    gemmbf) step gemmbf 300 python scripts/gemm_bench.py all 10 bf16 ;;
    pbf) step pbf 900 python -m pytest tests/test_gpu_parity.py -q -s -k bf16 ;;
    benchbf) step benchbf 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --dtype bf16 ;;
    attn) step attn 300 python scripts/attn_bench.py both ;;
    apaths) step apaths 300 python scripts/attn_paths.py ;;
    dcost) step dcost 300 python scripts/dropout_cost.py ;;
    stamps) step stamps 120 scripts/lab/attn_stamps ;;
    stamps0) K3M_ATTN_FWD_REG=0 step stamps0 120 scripts/lab/attn_stamps ;;
    pmcattn) step pmcattn 300 scripts/lab/pmc_attn.sh 0 att0 ;;
    tattn) step tattn 600 python -u -m pytest tests -m gpu -k "attn or attention" -x -q --timeout 300 --timeout-method thread ;;
    tbf) step tbf 600 python -m pytest tests/test_gpu_gemm_bf16.py -q ;;
    ddp2) step ddp2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --backend gloo --batch 16 ;;
    pmc) export TMPDIR=/tmp
         step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o run -- python scripts/gemm_bench.py "fwd ffn1 gelu" 5
         step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o run -- python scripts/gemm_bench.py "fwd ffn1 gelu" 5 ;;
    data) step data 400 python -u -m pytest tests/test_gpu_data.py -x -v --timeout 120 --timeout-method thread ;;
    ft) step ft 600 python -u -m pytest tests/test_gpu_finetune.py -x -v --timeout 300 --timeout-method thread ;;
    bft) step bft 600 python scripts/bench_finetune.py --steps 10 --warmup 3 ;;
    pft) export TMPDIR=/tmp; step pft 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pft -o run -- python scripts/bench_finetune.py --steps 3 --warmup 1 --no-cpu-baseline ;;
    bdata) step bdata 300 python scripts/bench_data.py ;;
    pdata) export TMPDIR=/tmp; step pdata 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pdata -o run -- python scripts/bench_data.py --reps 50 ;;
    pmcdata) export TMPDIR=/tmp
         step pmcd_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcd_fetch -o run -- python scripts/bench_data.py --reps 20
         step pmcd_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmcd_write -o run -- python scripts/bench_data.py --reps 20 ;;
    flash) step flash 400 python -u -m pytest tests/test_gpu_gemm_bf16.py -k flash -q --timeout 120 --timeout-method thread ;;
    rccl) step rccl 900 python -u -m pytest tests/test_gpu_rccl.py -v -s --timeout 300 --timeout-method thread ;;
    standin) step standin 300 python -u -m pytest tests/test_gpu_dropin.py -q --timeout 200 --timeout-method thread ;;
    abkm) step abkm 900 scripts/ab_env.sh K3M_FLASH_BWD_KM "0 1" 3 --config 3 --steps 10 --warmup 4 ;;
    b16lab) for r in 1 2; do for lab in 0 1 2 3; do
              K3M_B16_LAB=$lab step b16lab_${lab}_$r 300 python scripts/gemm_bench.py all 20 bf16; done; done ;;
    tmode) step tmode 600 python -u -m pytest tests/test_gpu_train_mode_parity.py -v --timeout 300 --timeout-method thread ;;
    prof32) export TMPDIR=/tmp; step prof32 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof32 -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
    dual) step dualbit 400 python -u -m pytest tests/test_gpu_gemm_b16_dual.py -v --timeout 300 --timeout-method thread
          K3M_B16_DUAL=1 step dualbig 600 python -u -m pytest tests/test_gpu_gemm_b16_big.py tests/test_gpu_gemm_bf16.py -q --timeout 300 --timeout-method thread
          for d in 0 1; do K3M_B16_DUAL=$d step dualgemm_$d 300 python scripts/gemm_bench.py all 20 bf16; done
          step abdual 900 scripts/ab_env.sh K3M_B16_DUAL "0 1" 3 --config 3 --steps 10 --warmup 4 ;;
    dualbit) step dualbit 400 python -u -m pytest tests/test_gpu_gemm_b16_dual.py -v --timeout 300 --timeout-method thread ;;
    abdual2) step abdual2 900 scripts/ab_env.sh K3M_B16_DUAL "0 2" 3 --config 3 --steps 10 --warmup 4 ;;
    attnbf) step attnbf 300 python scripts/attn_bench.py bf16 ;;
    attn32) step attn32 300 python scripts/attn_bench.py fp32 ;;
    abopt) step abopt3 900 scripts/ab_env.sh K3M_OPT_OVERLAP "0 1" 3 --config 3 --steps 10 --warmup 4
           step abopt2 900 scripts/ab_env.sh K3M_OPT_OVERLAP "0 1" 2 --config 2 --steps 8 --warmup 4 ;;
    logiterr) step logiterr 400 python scripts/bf16_logit_errors.py gpurun_out/r4_bf16_logit_errors.json ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
