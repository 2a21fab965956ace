# gpu_r4b.sh -- round-4: the split2h GEMM tests, the split2h probe, the GPU suite (failures listed,
# not stopping at the first), the default and split2h benches, the shard step with the modelled collective
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3f.py -q -rf -k split2h --timeout 120 --timeout-method thread -s > $O/x3f_split2h.log 2>&1
echo "x3f exit $?" >> $O/x3f_split2h.log
grep -q "Fatal\|core dumped\|Segmentation" $O/x3f_split2h.log && exit 1
timeout -k 10 300 python -u tools/h2_probe.py > $O/h2_probe.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --maxfail=40 --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/gpu_tests.log
grep -q "Fatal\|core dumped\|Segmentation" $O/gpu_tests.log && exit 1
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 400 python bench.py --no-cpu-baseline --precision split2h > $O/bench_split2h.json 2> $O/bench_split2h.err || exit 1
timeout -k 10 300 python -u tools/shard_model.py 0 300 150 > $O/shard_model.txt 2>&1
echo done
