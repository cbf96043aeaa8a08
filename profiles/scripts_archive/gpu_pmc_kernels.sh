#!/bin/bash
# One rocprofv3 --pmc pass (8 SQ counters + GRBM_GUI_ACTIVE, counters only) over scripts/pmc_kernels.py.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p "$R/gpurun_out/pmck"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE -d /tmp/pmck -o k --output-format csv -- python3 "$R/scripts/pmc_kernels.py" > "$R/gpurun_out/pmck/k.log" 2>&1
rc=$?
find /tmp/pmck -name "*counter_collection.csv" -exec cp {} "$R/gpurun_out/pmck/" \;
exit $rc
