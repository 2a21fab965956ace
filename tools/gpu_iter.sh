# gpu_iter.sh TAG -- one iteration on the GPU: the update/shard parity tests, shard step times and
# the default bench line (outputs under gpurun_out/TAG/)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-iter}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_update.py tests/test_gpu_shard.py tests/test_gpu_fullbatch.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/shard_step.py 25 13 7 > $O/shard_step.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
echo done
