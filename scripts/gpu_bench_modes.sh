#!/bin/bash
# One gpurun call: headline bench over TCP (2 / 4 API workers), the mixed config-#5 stream and the
# decode GEMM plan.  Each GPU step has its own time limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
S=${BENCH_STEPS:-20}; W=${BENCH_WARMUP:-5}
timeout -k 10 600 python bench.py --steps $S --warmup $W --transport tcp --api-workers 2 --client-procs 2 > gpurun_out/bench_tcp_w2.log 2>&1 && \
timeout -k 10 600 python bench.py --steps $S --warmup $W --transport tcp --api-workers 4 --client-procs 3 > gpurun_out/bench_tcp_w4.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --mix > gpurun_out/bench_mix_asgi.log 2>&1 && \
timeout -k 10 600 python scripts/autotune_report.py 128 256 > gpurun_out/autotune_report.log 2>&1
rc=$?
echo "exit=$rc"
for f in gpurun_out/bench_tcp_w2.log gpurun_out/bench_tcp_w4.log gpurun_out/bench_mix_asgi.log; do tail -1 $f; done
exit $rc
