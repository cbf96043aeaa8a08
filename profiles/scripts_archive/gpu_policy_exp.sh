#!/bin/bash
# Scheduling-policy experiment: synchronized waves (default) vs a de-phased closed loop with
# every-step admission (mixed prefill+decode steps), plus the 2-rank DP path on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/pol_default.log 2>&1 && \
KA_PREFILL_MIN_FRAC=0 KA_PREFILL_MAX_WAIT_MS=0 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --ramp-s 0.25 > gpurun_out/pol_mixed_ramp.log 2>&1 && \
KA_PREFILL_MIN_FRAC=0.05 KA_PREFILL_MAX_WAIT_MS=2 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --ramp-s 0.25 > gpurun_out/pol_mixed_ramp05.log 2>&1 && \
BENCH_DEVICE=cuda:0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --concurrency 128 > gpurun_out/pol_dp2_onegpu.log 2>&1
rc=$?
for f in gpurun_out/pol_*.log; do echo "== $f"; grep -o '"value": [0-9.]*\|"p50_ms": [0-9.]*\|"decode_ms_per_step": [0-9.]*\|"prefill_ms_per_step": [0-9.]*\|"decode_steps": [0-9]*\|"prefill_steps": [0-9]*\|"n_gpus": [0-9]*' $f | tr '\n' ' '; echo; done
exit $rc
