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
run_prof() { cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 ${BENCH_ARGS} > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1; cd "$GRAFT_REPO_ROOT"; }
case "$STEP" in
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
