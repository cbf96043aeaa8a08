#!/bin/bash
# Round 5, GPU call i: what bounds the M = 256 decode GEMMs (csrc/gemm_mfma.hip ring kernels)?
# Ablation builds (tools/gemm_bench_a{1,2,3,4,8}: no weight DMA / no X DMA / neither / no MFMA / no
# fragment reads; wrong results on purpose) of the planned configurations, and 32-deep-k ring
# configurations (ids 20-23, -DKA_GM_EXTRA) against the planned ones and rocBLAS.
set -o pipefail
O=gpurun_out/r5i
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
PLANNED="256,6144,4096,2,4,2 256,4096,4096,12,4,2 256,4096,14336,2,8,2 256,28672,4096,2,1,3"
for v in x a1 a2 a3 a4 a8; do
  echo "== $v" >> $O/abl.log
  timeout -k 10 120 tools/gemm_bench_$v $PLANNED >> $O/abl.log 2>&1
  rc=$?; [ $rc -eq 0 ] || stop $v $rc
done
X=""
for s in 256,6144,4096 256,4096,4096 256,4096,14336; do
  X="$X $s,-1,1,0"
  for c in 2 12 20 21 22 23; do for sp in 2 4 8; do X="$X $s,$c,$sp,2"; done; done
done
X="$X 256,28672,4096,-1,1,0 256,28672,4096,2,1,3 256,28672,4096,20,1,3 256,28672,4096,21,1,3 256,28672,4096,23,1,3 256,28672,4096,20,2,2"
for r in 1 2; do
  echo "== cfg sweep rep $r" >> $O/cfg.log
  timeout -k 10 300 tools/gemm_bench_x $X >> $O/cfg.log 2>&1
  rc=$?; [ $rc -eq 0 ] || stop cfg$r $rc
done
echo ALL DONE
