set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/it3
mkdir -p $O
timeout -k 10 200 python -u tools/shard_step.py 7 6 > $O/shard_default.txt 2>&1 || exit 1
MTSAC_X3F_MIN_TILES=32 timeout -k 10 200 python -u tools/shard_step.py 7 6 > $O/shard_min32.txt 2>&1 || exit 1
MTSAC_X3F_MIN_TILES=32 timeout -k 10 600 python -u -m pytest tests/test_gpu_fullbatch.py tests/test_gpu_shard.py -x -q --timeout 300 --timeout-method thread > $O/tests_min32.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/tests_min32.log
exit $rc
