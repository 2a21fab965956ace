#!/bin/bash
# sums.sh TAG "ARGS"... -- serialised per-kernel step sums (rocprofv3 kernel trace, tools/kernel_sums.py) of
# tools/shard_prof.py ARGS (T_local T W precision), one output file per argument set
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for A in "$@"; do
  N=$(echo $A | tr ' ' '_')
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt$N -o run -- python $R/tools/shard_prof.py $A > $O/kt$N.log 2>&1 || exit 1
  python $R/tools/kernel_sums.py $O/kt$N/run_kernel_trace.csv 45 > $O/sums_$N.txt || exit 1
  rm -rf $O/kt$N
done
echo done
