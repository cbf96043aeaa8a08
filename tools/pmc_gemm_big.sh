#!/bin/bash
# PMC passes over tools/gemm_big_bench (one rocprofv3 --pmc run per counter set; run from the repo root
# on the GPU box).  Writes counter CSVs + a per-kernel summary to gpurun_out/pmc_big/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; export TMPDIR=/tmp
CASES="${CASES:-4096,28672,4096,0}"
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"
OUT=$R/gpurun_out/pmc_big; mkdir -p $OUT
cd /tmp
for i in 1 2 3; do
  eval P=\$P$i
  GB_ROUNDS=1 timeout -s KILL 90 rocprofv3 --pmc $P -d /tmp/pmcb$i -o p$i --output-format csv -- $R/tools/gemm_big_bench $CASES > $OUT/run$i.log 2>&1 || exit $?
  find /tmp/pmcb$i -name "*counter_collection.csv" -exec cp {} $OUT/p$i.csv \;
done
python3 - "$OUT" <<'PY'
import csv, sys, collections, os
out = sys.argv[1]
for i in (1, 2, 3):
    path = os.path.join(out, f"p{i}.csv")
    if not os.path.exists(path):
        print("missing", path); continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        agg[r["Kernel_Name"][:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in agg.items():
        if "fill" in k or "ref_kernel" in k: continue
        print(k)
        print("   " + "  ".join(f"{c}={sum(v)/len(v):.3g}" for c, v in sorted(d.items())))
PY
