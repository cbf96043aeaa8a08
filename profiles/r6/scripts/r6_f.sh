#!/bin/bash
# Round 6, call f: the Llama-3-70B TP = 8 rank's plans re-tuned with the O / down partials fed to the
# collective (KA_GEMM_PLAN=write), then virtual-rank decode steps: split-K into the collective on / off,
# and the round-5 kernels (counted waits, tools/lib_counted) with it off; the parity tests once more.
set -o pipefail
O=gpurun_out/r6f
mkdir -p $O/tuned
KA_GEMM_PLAN=write PLAN_COPY_TO=$O/tuned timeout -k 10 600 python -u scripts/bench_virtual_rank.py --model llama3-70b --tp 8 --buckets 1,2,4,8,16,32,64,128,256 > $O/vrank70_write.log 2>&1; echo "write rc=$?"; tail -3 $O/vrank70_write.log
cp ai_agent_kubectl_amd/ops/tuned/gemm_plan_mi355x.json $O/tuned/gemm_plan_mi355x.json
for rep in 1 2; do
KA_TP_SPLITK_NORM=1 timeout -k 10 300 python -u scripts/bench_virtual_rank.py --model llama3-70b --tp 8 --buckets 1,8,64,256 > $O/vrank70_on_$rep.log 2>&1; echo "on rc=$?"; grep "decode graph" $O/vrank70_on_$rep.log
KA_TP_SPLITK_NORM=0 timeout -k 10 300 python -u scripts/bench_virtual_rank.py --model llama3-70b --tp 8 --buckets 1,8,64,256 > $O/vrank70_off_$rep.log 2>&1; echo "off rc=$?"; grep "decode graph" $O/vrank70_off_$rep.log
KA_TP_SPLITK_NORM=0 KA_HIP_LIB_DIAG=1 KA_HIP_LIB=tools/lib_counted/libkagent_hip.so timeout -k 10 300 python -u scripts/bench_virtual_rank.py --model llama3-70b --tp 8 --buckets 1,8,64,256 > $O/vrank70_r5kernels_$rep.log 2>&1; echo "r5 rc=$?"; grep "decode graph" $O/vrank70_r5kernels_$rep.log
done
timeout -k 10 900 python -u -m pytest tests/test_model_full_depth_gpu.py -v -s --timeout 600 --timeout-method thread > $O/full_depth.log 2>&1
echo "full depth rc=$?"; grep -E "mean greedy|repeats|passed|failed" $O/full_depth.log | tail -12
