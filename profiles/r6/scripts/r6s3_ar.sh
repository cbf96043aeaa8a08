#!/bin/bash
# Round 6 session 3: peer reads batched in the one-shot all-reduce (+ RMSNorm) and the persistent
# kernel's in-kernel all-reduce: the collective / TP tests (2 ranks sharing the GPU), the persistent
# decode tests, then the 2-rank persistent TP step and the collective's graph timing.
set -o pipefail
O=gpurun_out/r6s3_ar
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_custom_allreduce_gpu.py tests/test_tp_single_gpu.py tests/test_model_gpu.py -k "allreduce or tp or persistent or collective" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -1 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u scripts/bench_tp_persistent_2rank.py --model llama3-70b-8l --reps 50 > $O/tp2_two_ranks.log 2>&1
rc=$?; echo "tp2 rc $rc"; grep -i "ms" $O/tp2_two_ranks.log | tail -4; exit $rc
