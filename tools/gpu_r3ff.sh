# gpu_r3ff.sh -- input-layer weight grad on k-major planes: parity subset, A/B shard steps, C1 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3ff
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_update.py tests/test_gpu_fullbatch.py tests/test_gpu_shard.py tests/test_gpu_multiprocess.py tests/test_gpu_trainer.py -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/shard_step.py 50 13 7 > $O/shard_steps_planes.txt 2>&1 || exit 1
MTSAC_INPUT_WGRAD=0 timeout -k 10 300 python -u tools/shard_step.py 50 13 7 > $O/shard_steps_onthefly.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload mt10_w400 --no-cpu-baseline > $O/bench_c1.json 2> $O/bench_c1.err || exit 1
MTSAC_INPUT_WGRAD=0 timeout -k 10 300 python bench.py --workload mt10_w400 --no-cpu-baseline > $O/bench_c1_otf.json 2> $O/bench_c1_otf.err || exit 1
echo done
