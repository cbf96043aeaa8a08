#!/bin/bash
# One gpurun call: GPU tests, smoke, short bench, rocprof kernel stats.  Every GPU step has its own
# time limit and the steps are chained so the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEP="${1:-all}"
run_tests() { timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; }
run_smoke() { timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; }
run_bench() { timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-5} --warmup ${BENCH_WARMUP:-2} ${BENCH_ARGS} > gpurun_out/bench.log 2>&1; }
run_prof() { rm -rf /tmp/ka_prof && cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/ka_prof -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 ${BENCH_ARGS} > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1; rc=$?; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof && find /tmp/ka_prof -name "*stats.csv" -exec cp {} gpurun_out/prof/ \; ; python scripts/trace_busy.py /tmp/ka_prof --window ${TRACE_WINDOW:-2.0} > gpurun_out/trace_busy.txt 2>&1; return $rc; }
run_cprof() { KA_PROFILE_ENGINE=gpurun_out/cprof_engine.txt KA_PROFILE_API=gpurun_out/cprof_api.txt timeout -k 10 600 python bench.py --steps 3 --warmup 1 ${BENCH_ARGS} > gpurun_out/bench_cprof.log 2>&1; }
run_gemm() { timeout -k 10 600 python scripts/bench_gemm.py > gpurun_out/bench_gemm.log 2>&1; }
run_ktest() { timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider > gpurun_out/pytest_kernels.log 2>&1; }
run_sweep() { for c in ${SWEEP:-64 128 256}; do timeout -k 10 600 python bench.py --steps 4 --warmup 2 --concurrency $c ${BENCH_ARGS} > gpurun_out/bench_c$c${TAG}.log 2>&1 || return 1; done; }
run_tunab() { KA_TUNABLEOP=1 KA_TUNABLEOP_WRITE=1 KA_TUNABLEOP_FILE=gpurun_out/tunableop_results.csv timeout -k 10 900 python bench.py --steps 4 --warmup 2 --concurrency ${C:-256} > gpurun_out/bench_tunable.log 2>&1; }
run_big() { timeout -k 10 1200 python scripts/bigmodel_check.py ${BIG_MODELS} > gpurun_out/bigmodel.log 2>&1; }
run_mixed() { timeout -k 10 600 python scripts/bench_service.py mixed --backend engine --concurrency ${C:-64} --seconds 20 > gpurun_out/mixed.log 2>&1; }
run_phase() { timeout -k 10 600 python scripts/phase_profile.py --concurrency ${C:-256} > gpurun_out/phase_profile.log 2>&1; }
case "$STEP" in
  phase) run_phase ;;
  policy) SWEEP="256" TAG=_p025 run_sweep && KA_PREFILL_MIN_FRAC=0 KA_PREFILL_MAX_WAIT_MS=0 SWEEP="256 384" TAG=_p0 run_sweep && KA_PREFILL_MIN_FRAC=0.1 KA_PREFILL_MAX_WAIT_MS=5 SWEEP="256" TAG=_p01 run_sweep && KA_SPLIT_MIXED_ATTN=0 KA_PREFILL_MIN_FRAC=0 KA_PREFILL_MAX_WAIT_MS=0 SWEEP="256" TAG=_p0nosplit run_sweep ;;
  big) run_big ;;
  mixed) run_mixed ;;
  bigmixed) run_mixed && run_big ;;
  tunab) run_tunab && C=256 run_sweep ;;
  sweep) run_sweep ;;
  modes) SWEEP="128 256" run_sweep && SWEEP="128 256" TAG=_inproc BENCH_ARGS="--in-process" run_sweep && C=64 run_mixed ;;
  testsweep) run_tests && run_sweep ;;
  gemm) run_ktest && run_gemm ;;
  gemmbench) run_ktest && run_gemm && run_tests && run_bench ;;
  cprof) run_cprof ;;
  profall) run_bench && run_prof && run_cprof ;;
  tests) run_tests ;;
  smoke) run_smoke ;;
  bench) run_bench ;;
  prof) run_prof ;;
  all) run_tests && run_smoke && run_bench ;;
  benchprof) run_bench && run_prof ;;
esac
rc=$?
echo "exit=$rc"
tail -5 gpurun_out/*.log
exit $rc
