# gpu_r3t.sh -- in-launch finish v2 (sc1 slabs, prefetch; x3p reduce): microbench, tests, shard A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3t
mkdir -p $O
timeout -k 10 120 python -u tools/fin_bench.py > $O/fin_bench.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_x3f.py tests/test_gpu_x3p.py tests/test_gpu_shard.py tests/test_gpu_fullbatch.py -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/shard_step.py 50 25 13 7 > $O/shard_steps_fin.txt 2>&1 || exit 1
MTSAC_X3F_FIN=0 MTSAC_X3P_FIN=0 timeout -k 10 300 python -u tools/shard_step.py 25 13 7 > $O/shard_steps_nofin.txt 2>&1 || exit 1
MTSAC_X3F_FIN=0 timeout -k 10 300 python -u tools/shard_step.py 13 7 > $O/shard_steps_x3pfin_only.txt 2>&1 || exit 1
echo done
