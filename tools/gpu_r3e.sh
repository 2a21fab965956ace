# gpu_r3e.sh -- bf16 row tiles 48/80/208/400 (no split-K): kernel tests, drift bound, bf16 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_x3f.py tests/test_gpu_x3p.py tests/test_gpu_fullbatch.py tests/test_gpu_update.py -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --precision bf16 --no-cpu-baseline > $O/bench_s3_bf16.json 2> $O/bench_s3_bf16.err || exit 1
timeout -k 10 300 python bench.py --precision bf16 --workload mt10_w2048 --no-cpu-baseline > $O/bench_c2_bf16.json 2> $O/bench_c2_bf16.err || exit 1
timeout -k 10 300 python bench.py --workload mt10_w2048 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || exit 1
timeout -k 10 300 python bench.py --workload mt10_w400 --no-cpu-baseline > $O/bench_c1.json 2> $O/bench_c1.err || exit 1
echo done
