# gpu_r3j.sh -- one-launch step tail (alpha + finish kernels), 112-row split-K tile for task shards
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3j
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/shard_step.py 50 25 13 7 > $O/shard_steps.txt 2>&1 || exit 1
MTSAC_X3F_SPLIT_BM=128 timeout -k 10 200 python tools/shard_step.py 13 7 > $O/shard_steps_bm128.txt 2>&1 || exit 1
MTSAC_X3F_SPLIT_BM=208 timeout -k 10 200 python tools/shard_step.py 13 7 > $O/shard_steps_bm208.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/kt_w400 -o run -- python $GRAFT_REPO_ROOT/tools/shard_prof.py 10 10 400 > $GRAFT_REPO_ROOT/$O/kt_w400.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/kt_t7 -o run -- python $GRAFT_REPO_ROOT/tools/shard_prof.py 7 > $GRAFT_REPO_ROOT/$O/kt_t7.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python tools/kernel_sums.py $O/kt_w400/run_kernel_trace.csv 60 > $O/sums_w400.txt || exit 1
python tools/kernel_sums.py $O/kt_t7/run_kernel_trace.csv 60 > $O/sums_t7.txt || exit 1
rm -rf $O/kt_w400 $O/kt_t7
timeout -k 10 300 python bench.py --workload mt10_w400 --no-cpu-baseline > $O/bench_c1.json 2> $O/bench_c1.err || exit 1
echo done
