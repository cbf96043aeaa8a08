#!/bin/bash
# PMC pass over the prefill attention microbenchmark (chunk-resident kernel).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p "$R/gpurun_out/pmcpa"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d /tmp/pmcpa -o pa --output-format csv -- python3 "$R/scripts/bench_prefill_attn.py" > "$R/gpurun_out/pmcpa/pa.log" 2>&1
rc=$?
find /tmp/pmcpa -name "*counter_collection.csv" -exec cp {} "$R/gpurun_out/pmcpa/" \;
exit $rc
