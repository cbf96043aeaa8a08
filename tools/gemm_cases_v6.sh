#!/bin/bash
# Decode shapes (M = 256 and 128): 64-row weight tiles (cfgs 6, 20-25) vs the current plan and rocBLAS.
B=tools/gemm_bench
P=""
for shape in 256,28672,4096 128,28672,4096; do
  P="$P $shape,-1,1,0 $shape,2,1,0 $shape,2,1,3"
  for c in 6 20 21 22 23 24 25; do P="$P $shape,$c,1,0 $shape,$c,1,3"; done
done
for shape in 256,6144,4096 256,4096,4096 256,4096,14336 128,6144,4096 128,4096,4096 128,4096,14336; do
  P="$P $shape,-1,1,0"
  for c in 4 6 20 21 22 23 24 25; do for sp in 1 2 4 8; do P="$P $shape,$c,$sp,2"; done; done
done
P="$P 256,128256,4096,-1,1,0 256,128256,4096,3,1,0 256,128256,4096,6,1,0 256,128256,4096,20,1,0 256,128256,4096,21,1,0 256,128256,4096,22,1,0"
$B $P
