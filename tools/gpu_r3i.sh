# gpu_r3i.sh -- fused optimizer launches + producer-written input planes + static row lists
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3i
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/shard_step.py 50 25 13 7 > $O/shard_steps.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/kt_w400 -o run -- python $GRAFT_REPO_ROOT/tools/shard_prof.py 10 10 400 > $GRAFT_REPO_ROOT/$O/kt_w400.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python tools/kernel_sums.py $O/kt_w400/run_kernel_trace.csv 60 > $O/sums_w400.txt || exit 1
rm -rf $O/kt_w400
timeout -k 10 300 python bench.py --workload mt10_w400 --no-cpu-baseline > $O/bench_c1.json 2> $O/bench_c1.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_s3.json 2> $O/bench_s3.err || exit 1
echo done
