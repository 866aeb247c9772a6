#!/bin/bash
# PMC passes over one attention shape: usage bash tools/pmc_attn.sh B n H hd bwd
set -o pipefail
export TMPDIR=/tmp
mkdir -p ${PMCDIR:-gpurun_out/pmca}
for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" "SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32 SQ_WAVES" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  tag=$(echo $ctr | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d ${PMCDIR:-gpurun_out/pmca}/$tag -o run -- python tools/attn_one.py "$@" > /dev/null 2>&1 || echo "fail $ctr"
done
python - <<'PY'
import csv, glob, collections, os
agg = collections.defaultdict(list)
for f in glob.glob(os.environ.get("PMCDIR", "gpurun_out/pmca") + "/*/*counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "attn" in r.get("Kernel_Name", ""):
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:28s} mean/dispatch = {sum(v)/len(v):.4g}  (n={len(v)})")
PY
