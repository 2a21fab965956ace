# gpu_r3a.sh -- round-3 iteration: the new / changed GPU tests (multi-process shard, producer-stream
# adds, DrQ at the benched batch, sharded hook buckets, update parity)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_drq.py tests/test_gpu_shard.py tests/test_gpu_update.py tests/test_gpu_fullbatch.py -v -s -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/tests.log
exit $rc
