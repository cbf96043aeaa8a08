#!/bin/bash
# Round 6 session 3: 2- vs 4-wave decode attention workgroups at B = 256 after the prologue changes.
set -o pipefail
O=gpurun_out/r6s3_nw
mkdir -p $O
timeout -k 10 300 python -u scripts/bench_decode_attn_ctx.py --ctx 65,121,131 > $O/nw2.log 2>&1 || exit 1
KA_DECODE_NW2_MIN_WGS=0 timeout -k 10 300 python -u scripts/bench_decode_attn_ctx.py --ctx 65,121,131 > $O/nw4.log 2>&1 || exit 1
grep -h "us$" $O/nw2.log $O/nw4.log
