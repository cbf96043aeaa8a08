#!/bin/bash
# Decode projection shapes (Llama-3-8B, M = 128 / 256): the autotuned gemm_mfma configurations
# against rocBLAS.  Build: see the header of tools/gemm_bench.hip (add -DGM_BSTAMPS for per-block
# timelines of the ring kernels).
B=${GEMM_BENCH:-tools/gemm_bench}
P=""
for M in 128 256; do
  P="$P $M,28672,4096,-1,1,0 $M,28672,4096,2,1,0 $M,28672,4096,2,1,3 $M,28672,4096,3,1,0 $M,28672,4096,19,2,2"
  for shape in $M,6144,4096 $M,4096,4096 $M,4096,14336; do
    P="$P $shape,-1,1,0"
    for c in 4 5 12 2; do for sp in 2 4 8; do P="$P $shape,$c,$sp,2"; done; done
  done
done
$B $P
