#!/bin/bash
# drq_kprof.sh TAG -- rocprofv3 kernel stats of 11 resident-batch DrQ-eps updates (tools/drq_prof.py)
set -o pipefail
TAG=${1:-drqprof}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$TAG -o run -- python $R/tools/drq_prof.py > $R/gpurun_out/$TAG.log 2>&1 || exit 1
python3 - "$R/gpurun_out/$TAG/run_kernel_stats.csv" <<'PY' | tee $R/gpurun_out/$TAG/summary.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
print("total us/step", round(sum(float(r["TotalDurationNs"]) for r in rows) / 11e3, 1))
for r in rows[:30]:
    print(round(float(r["TotalDurationNs"]) / 11e3, 1), r["Calls"], r["Name"][:100])
PY
