#!/bin/bash
# Two PMC passes (each in its own rocprofv3 run, --pmc only) over scripts/pmc_gemm.py.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p "$R/gpurun_out/pmc"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum -d /tmp/pmc1 -o p1 --output-format csv -- python3 "$R/scripts/pmc_gemm.py" > "$R/gpurun_out/pmc/p1.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum -d /tmp/pmc2 -o p2 --output-format csv -- python3 "$R/scripts/pmc_gemm.py" > "$R/gpurun_out/pmc/p2.log" 2>&1
rc=$?
find /tmp/pmc1 /tmp/pmc2 -name "*counter_collection.csv" -exec cp {} "$R/gpurun_out/pmc/" \; 2>/dev/null
ls -la "$R/gpurun_out/pmc/"
exit $rc
