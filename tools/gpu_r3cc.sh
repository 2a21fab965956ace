# gpu_r3cc.sh -- dbp finishing kernel v2: shard / full-batch parity, T7 step + kernel sums
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3cc
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullbatch.py tests/test_gpu_shard.py tests/test_gpu_update.py -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/shard_step.py 25 13 7 > $O/shard_steps.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/kt_t7 -o run -- python $GRAFT_REPO_ROOT/tools/shard_prof.py 7 > $GRAFT_REPO_ROOT/$O/kt_t7.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python tools/kernel_sums.py $O/kt_t7/run_kernel_trace.csv 60 > $O/sums_t7.txt || exit 1
rm -rf $O/kt_t7
echo done
