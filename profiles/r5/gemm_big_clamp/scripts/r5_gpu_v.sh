#!/bin/bash
# Round 5, GPU call v: gemm_big wrong rows with the clamp as the amplifier — does a pad after each
# vmcnt wait (c1n) or draining every wait to 0 (c1z) remove them?  Then the default library (distinct
# rows) on both shapes, and the gemm_mfma kernel tests after its distinct-row change.
set -o pipefail
O=gpurun_out/r5v
mkdir -p $O
stop() { echo "STOP after $1 (rc $2)"; exit $2; }
for v in c1 c1n c1z; do
  echo "== $v" >> $O/diag.log
  KA_HIP_LIB=ai_agent_kubectl_amd/ops/lib/variants/libkagent_hip_$v.so DIAG_SHAPES=4096x1152x4096 DIAG_REPS=40 \
    timeout -k 10 240 python -u profiles/r5/gemm_big_clamp/gb_wrong_rows_diag.py >> $O/diag.log 2>&1
  rc=$?; [ $rc -eq 0 ] || stop $v $rc
done
echo "== def" >> $O/diag.log
DIAG_SHAPES=4096x1152x4096,2944x6144x4096 DIAG_REPS=80 timeout -k 10 300 python -u profiles/r5/gemm_big_clamp/gb_wrong_rows_diag.py >> $O/diag.log 2>&1 || stop def $?
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "gm or mfma or ring" > $O/pytest_gm.log 2>&1 || stop pytest_gm $?
echo ALL DONE
