#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  tag=$(echo $ctr | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc/$tag -o run -- python tools/gemm_one.py "$@" > /dev/null 2>&1 || echo "fail $ctr"
done
python - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for f in glob.glob("gpurun_out/pmc/*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "gemm" in r.get("Kernel_Name", ""):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:28s} mean/dispatch = {sum(v)/len(v):.4g}  (n={len(v)})")
PY
