#!/bin/bash
# PMC passes over the GEMM harness (one rocprofv3 --pmc run per counter set; cd /tmp first)
set -o pipefail
R=$GRAFT_REPO_ROOT; export TMPDIR=/tmp; cd /tmp
CASES="${CASES:-8192,28672,4096,19,1,0 8192,28672,4096,-1,1,0 256,28672,4096,2,1,0 256,28672,4096,-1,1,0}"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum"
timeout -s KILL 90 rocprofv3 --pmc $P1 -d /tmp/pmc1 -o p1 --output-format csv -- $R/tools/gemm_bench $CASES > $R/gpurun_out/pmc1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc $P2 -d /tmp/pmc2 -o p2 --output-format csv -- $R/tools/gemm_bench $CASES > $R/gpurun_out/pmc2.log 2>&1
rc=$?
mkdir -p $R/gpurun_out/pmc; find /tmp/pmc1 /tmp/pmc2 -name "*counter_collection.csv" -exec cp {} $R/gpurun_out/pmc/ \; 2>/dev/null
exit $rc
