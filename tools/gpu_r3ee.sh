# gpu_r3ee.sh -- nontemporal tile-Adam stores: parity subset, T7 / T50 kernel sums
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3ee
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_update.py tests/test_gpu_fullbatch.py -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/tests.log
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/kt_t7 -o run -- python $GRAFT_REPO_ROOT/tools/shard_prof.py 7 > $GRAFT_REPO_ROOT/$O/kt_t7.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/kt_t50 -o run -- python $GRAFT_REPO_ROOT/tools/shard_prof.py 50 > $GRAFT_REPO_ROOT/$O/kt_t50.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python tools/kernel_sums.py $O/kt_t7/run_kernel_trace.csv 60 > $O/sums_t7.txt || exit 1
python tools/kernel_sums.py $O/kt_t50/run_kernel_trace.csv 60 > $O/sums_t50.txt || exit 1
rm -rf $O/kt_t7 $O/kt_t50
echo done
