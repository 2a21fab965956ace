# gpu_r3aa.sh -- TD target fused into the critic-loss head launch: GPU suite, C1 / S3 / T7, C1 timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3aa
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload mt10_w400 --no-cpu-baseline > $O/bench_c1.json 2> $O/bench_c1.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_s3.json 2> $O/bench_s3.err || exit 1
timeout -k 10 300 python -u tools/shard_step.py 7 > $O/shard_steps.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/kt_c1 -o run -- python $GRAFT_REPO_ROOT/tools/c1_timeline.py > $GRAFT_REPO_ROOT/$O/kt_c1.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python tools/step_timeline.py $O/kt_c1/run_kernel_trace.csv full > $O/c1_timeline.txt || exit 1
rm -rf $O/kt_c1
echo done
