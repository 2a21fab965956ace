# gpu_r4k.sh -- round-4: x3f epilogue with four 16-row blocks per barrier: GEMM tests, probe, S3 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4k
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_x3f.py tests/test_gpu_fullbatch.py -q -rf -x -k "x3f or full_batch_step or shard" --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/h2_probe.py > $O/h2_probe.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --precision split3 > $O/bench_split3.json 2> $O/bench_split3.err || exit 1
echo done
