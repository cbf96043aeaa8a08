#!/bin/bash
# Round 5, GPU call u: gemm_big wrong rows 56-63 — library variants (c1: rows past the end clamped to the
# last row, c1e: clamped + M0 set per LDS-DMA piece, def: distinct rows, e: distinct + M0 per piece).
set -o pipefail
O=gpurun_out/r5u
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
for v in c1 c1e def e; do
  echo "== $v" >> $O/diag.log
  KA_HIP_LIB=ai_agent_kubectl_amd/ops/lib/variants/libkagent_hip_$v.so DIAG_SHAPES=2944x6144x4096,4096x1152x4096 DIAG_REPS=40 \
    timeout -k 10 240 python -u profiles/r5/gemm_big_clamp/gb_wrong_rows_diag.py >> $O/diag.log 2>&1
  rc=$?; [ $rc -eq 0 ] || stop $v $rc
done
echo ALL DONE
