#!/bin/bash
# Round 5, GPU call w: gemm_big counted-vmcnt hazard — cost of draining the LDS-DMA waits.
#   def: counted vmcnt(16) at barrier #2 (current); vm0: every wait vmcnt(0);
#   db1: k-tile t + 1 waited for with vmcnt(0) at barrier #1, before t + 2's pieces (barrier #2 dropped)
# then the clamp amplifier with db1 (c1b) and db1 itself in the python alternating-shape diag.
set -o pipefail
O=gpurun_out/r5w
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
CASES="2944,6144,4096,0 4096,6144,4096,0 4096,4096,4096,0 4096,4096,14336,0 2944,28672,4096,3 4096,28672,4096,3 4096,1152,4096,0 4096,8192,8192,0 4096,57344,8192,3 4096,8192,28672,0"
for v in def vm0 db1 def db1; do
  echo "== $v" >> $O/perf.log
  GB_ROUNDS=5 timeout -k 10 300 tools/gemm_big_bench_$v $CASES >> $O/perf.log 2>&1
  rc=$?; [ $rc -le 1 ] || stop $v $rc
done
for v in c1b db1; do
  echo "== $v" >> $O/diag.log
  KA_HIP_LIB=ai_agent_kubectl_amd/ops/lib/variants/libkagent_hip_$v.so DIAG_SHAPES=4096x1152x4096,2944x6144x4096 DIAG_REPS=60 \
    timeout -k 10 300 python -u profiles/r5/gemm_big_clamp/gb_wrong_rows_diag.py >> $O/diag.log 2>&1
  rc=$?; [ $rc -eq 0 ] || stop $v $rc
done
echo ALL DONE
