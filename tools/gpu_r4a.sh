# gpu_r4a.sh -- round-4 first box: lane-divergence localisation (fresh child processes), the split2h
# gemm_x3f probe, then the GPU suite and the default bench as this round's baseline
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 300 python -u tools/lane_diverge.py 4 48 > $O/lane_diverge_wgrad_planes.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/lane_diverge.py 4 48 MTSAC_INPUT_WGRAD=0 > $O/lane_diverge_wgrad_fp32.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3f.py -x -q -rf -k split2h --timeout 120 --timeout-method thread -s > $O/x3f_split2h.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/h2_probe.py > $O/h2_probe.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
echo done
