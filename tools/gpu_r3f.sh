# gpu_r3f.sh -- bf16 tiles + narrow-trunk wgrad tiles + cross-step pipelined eager steps
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullbatch.py tests/test_gpu_x3f.py tests/test_gpu_x3p.py tests/test_gpu_update.py tests/test_gpu_shard.py tests/test_gpu_multiprocess.py tests/test_gpu_buffer_async.py tests/test_gpu_trainer.py -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/shard_step.py 50 25 13 7 > $O/shard_steps.txt 2>&1 || exit 1
MTSAC_NO_PIPELINE=1 timeout -k 10 300 python tools/shard_step.py 25 7 > $O/shard_steps_nopipe.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --precision bf16 --no-cpu-baseline > $O/bench_s3_bf16.json 2> $O/bench_s3_bf16.err || exit 1
timeout -k 10 300 python bench.py --precision bf16 --workload mt10_w2048 --no-cpu-baseline > $O/bench_c2_bf16.json 2> $O/bench_c2_bf16.err || exit 1
timeout -k 10 300 python bench.py --workload mt10_w2048 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || exit 1
timeout -k 10 300 python bench.py --workload mt10_w400 --no-cpu-baseline > $O/bench_c1.json 2> $O/bench_c1.err || exit 1
timeout -k 10 300 python bench.py --workload mt50_w400 --no-cpu-baseline > $O/bench_s4.json 2> $O/bench_s4.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_s3.json 2> $O/bench_s3.err || exit 1
echo done
