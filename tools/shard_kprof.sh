# shard_kprof.sh TAG TL... -- serialised per-kernel step sums of task shards (rocprofv3 kernel trace)
set -o pipefail
TAG=$1; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for TL in "$@"; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt$TL -o run -- python $R/tools/shard_prof.py $TL > $O/kt$TL.log 2>&1 || exit 1
  python $R/tools/kernel_sums.py $O/kt$TL/run_kernel_trace.csv 45 > $O/sums_$TL.txt || exit 1
  rm -rf $O/kt$TL
done
echo done
