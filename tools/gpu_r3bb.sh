# gpu_r3bb.sh -- batched tile-Adam loads, lazy segment events: parity subset, T7 / S3 kernel sums, benches
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3bb
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/shard_step.py 50 7 > $O/shard_steps.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_s3.json 2> $O/bench_s3.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/kt_t7 -o run -- python $GRAFT_REPO_ROOT/tools/shard_prof.py 7 > $GRAFT_REPO_ROOT/$O/kt_t7.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/kt_t50 -o run -- python $GRAFT_REPO_ROOT/tools/shard_prof.py 50 > $GRAFT_REPO_ROOT/$O/kt_t50.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python tools/kernel_sums.py $O/kt_t7/run_kernel_trace.csv 60 > $O/sums_t7.txt || exit 1
python tools/kernel_sums.py $O/kt_t50/run_kernel_trace.csv 60 > $O/sums_t50.txt || exit 1
rm -rf $O/kt_t7 $O/kt_t50
echo done
