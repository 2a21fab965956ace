# gpu_r3dd.sh -- 8 rows per wave in the policy / action-grad heads: parity subset, S3 kernel sums, benches
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3dd
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullbatch.py tests/test_gpu_update.py tests/test_gpu_trainer.py -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_s3.json 2> $O/bench_s3.err || exit 1
timeout -k 10 300 python bench.py --workload atari_drq --no-cpu-baseline > $O/bench_drq.json 2> $O/bench_drq.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/kt_t50 -o run -- python $GRAFT_REPO_ROOT/tools/shard_prof.py 50 > $GRAFT_REPO_ROOT/$O/kt_t50.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python tools/kernel_sums.py $O/kt_t50/run_kernel_trace.csv 60 > $O/sums_t50.txt || exit 1
rm -rf $O/kt_t50
echo done
