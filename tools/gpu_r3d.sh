# gpu_r3d.sh -- tall bf16 gemm_x3f tile: kernel tests, bf16 drift bound, bf16 benches (S3, C2)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_x3f.py tests/test_gpu_fullbatch.py -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --precision bf16 --no-cpu-baseline > $O/bench_s3_bf16.json 2> $O/bench_s3_bf16.err || exit 1
timeout -k 10 300 python bench.py --precision bf16 --workload mt10_w2048 --no-cpu-baseline > $O/bench_c2_bf16.json 2> $O/bench_c2_bf16.err || exit 1
echo done
