# gpu_r4a.sh -- round-4 first box: lane-divergence localisation (fresh child processes), the split2h
# probes, the GPU suite (failures listed, not stopping at the first), the default and split2h benches
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 300 python -u tools/lane_diverge.py 3 48 > $O/lane_diverge_wgrad_planes.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3f.py -x -q -rf -k split2h --timeout 120 --timeout-method thread -s > $O/x3f_split2h.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/h2_probe.py > $O/h2_probe.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --maxfail=40 --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/gpu_tests.log
grep -q "Fatal\|core dumped\|Segmentation" $O/gpu_tests.log && exit 1
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 400 python bench.py --no-cpu-baseline --precision split2h > $O/bench_split2h.json 2> $O/bench_split2h.err
echo done
