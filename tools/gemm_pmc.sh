#!/bin/bash
# PMC passes (one rocprofv3 run per counter group) over tools/gemm_one.py ARGS; summaries to
# gpurun_out/$TAG/.  usage: tools/gemm_pmc.sh TAG which epi E M N K iters
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU" \
           "TA_BUSY_sum TA_TA_BUSY_sum TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run -- python $R/tools/gemm_one.py "$@" > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; }
done
python - "$O" <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
tot = collections.defaultdict(float); n = collections.defaultdict(int)
for f in glob.glob(O + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "gemm_x3" not in r["Kernel_Name"]:
            continue  # fills / splits of the harness
        k = r["Counter_Name"]; tot[k] += float(r["Counter_Value"]); n[k] += 1
disp = max(n.values()) if n else 1
with open(O + "/summary.txt", "w") as out:
    for k in sorted(tot):
        line = f"{k:28s} mean/dispatch {tot[k] / max(n[k], 1):.4g}  (dispatch rows {n[k]})"
        print(line); out.write(line + "\n")
PY
