#!/bin/bash
# Prefill SwiGLU GEMM: kernel + model GPU tests, then ASGI bench A/B (fused vs hipBLASLt + silu_mul),
# interleaved.  Every GPU step has its own time limit; the first failure ends the call.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  -k "swiglu or lm_head" tests/test_model_gpu.py > gpurun_out/swiglu_tests.log 2>&1 || { tail -40 gpurun_out/swiglu_tests.log; exit 1; }
tail -2 gpurun_out/swiglu_tests.log
for r in 1 2; do for v in 1 0; do
  KA_PREFILL_SWIGLU=$v timeout -k 10 300 python bench.py --transport asgi --steps 10 --warmup 3 > gpurun_out/bench_swiglu${v}_r$r.log 2>&1 || exit 1
  echo "swiglu=$v rep$r"; tail -1 gpurun_out/bench_swiglu${v}_r$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); x=d['detail']; print(d['value'], d['p50_ms'], x.get('decode_ms_per_step'), x.get('prefill_ms_per_step'))"
done; done
