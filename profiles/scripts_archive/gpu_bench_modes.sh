#!/bin/bash
# One gpurun call: the headline bench at the driver's steps/warmup in every transport / load mode the
# docs quote.  Each GPU step has its own time limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/modes
S=${BENCH_STEPS:-20}; W=${BENCH_WARMUP:-5}
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" > gpurun_out/modes/$name.log 2>&1 || { echo "FAILED: $name"; tail -5 gpurun_out/modes/$name.log; exit 1; }
  echo "$name: $(tail -1 gpurun_out/modes/$name.log)"
}
run asgi_c256 --steps $S --warmup $W
run tcp_w2 --steps $S --warmup $W --transport tcp --api-workers 2 --client-procs 2
run tcp_w4 --steps $S --warmup $W --transport tcp --api-workers 4 --client-procs 3
run asgi_varlen --steps $S --warmup $W --variable-len
run open_poisson_900 --steps 10 --warmup 3 --load open --rate 900
run mix --steps 10 --warmup 3 --mix
run asgi_c1 --steps 10 --warmup 3 --concurrency 1
