set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/it2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_x3f.py tests/test_gpu_update.py tests/test_gpu_shard.py tests/test_gpu_fullbatch.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/shard_step.py 13 7 6 > $O/shard_model.txt 2>&1 || exit 1
MTSAC_X3F_SPLIT_BM=208 timeout -k 10 200 python -u tools/shard_step.py 13 7 6 > $O/shard_208.txt 2>&1 || exit 1
MTSAC_X3F_SPLIT_BM=128 timeout -k 10 200 python -u tools/shard_step.py 13 7 6 > $O/shard_128.txt 2>&1 || exit 1
echo done
