#!/bin/bash
# Round 6 session 3: B = 256 fused decode attention time against the context length (chunks per wave).
set -o pipefail
O=gpurun_out/r6s3_attn
mkdir -p $O
timeout -k 10 300 python -u scripts/bench_decode_attn_ctx.py > $O/ctx_default.log 2>&1
rc=$?; echo "default rc $rc"; [ $rc -eq 0 ] || exit $rc
KA_DECODE_NW2_MIN_WGS=0 timeout -k 10 300 python -u scripts/bench_decode_attn_ctx.py > $O/ctx_nw4.log 2>&1
rc=$?; echo "nw4 rc $rc"; exit $rc
