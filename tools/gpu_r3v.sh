# gpu_r3v.sh -- 256x128 k16 weight grads at shard / MT10 sizes: tests, shard steps, C1 / S4 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3v
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_x3p.py tests/test_gpu_shard.py tests/test_gpu_fullbatch.py tests/test_gpu_update.py -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/shard_step.py 50 25 13 7 > $O/shard_steps.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload mt10_w400 --no-cpu-baseline > $O/bench_c1.json 2> $O/bench_c1.err || exit 1
timeout -k 10 300 python bench.py --workload mt50_w400 --no-cpu-baseline > $O/bench_s4.json 2> $O/bench_s4.err || exit 1
echo done
