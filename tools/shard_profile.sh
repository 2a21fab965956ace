# shard_profile.sh TAG T_local -- per-shard step times and a serialised kernel breakdown of one shard
set -o pipefail
TAG=${1:-shard}; TL=${2:-7}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 200 python -u tools/shard_step.py 50 10 7 6 > $O/shard_step.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python $R/tools/shard_prof.py $TL > $O/kt.log 2>&1 || exit 1
python $R/tools/kernel_sums.py $O/kt/run_kernel_trace.csv 45 > $O/sums_$TL.txt
python $R/tools/step_timeline.py $O/kt/run_kernel_trace.csv full > $O/timeline_$TL.txt
rm -rf $O/kt
echo done
