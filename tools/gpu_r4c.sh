# gpu_r4c.sh -- round-4: split2h GEMM tests with the plane diagnostics, DrQ on f32-MFMA convs (parity both
# ways, bench both ways, kernel stats both ways)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3f.py -q -rf -k split2h --timeout 120 --timeout-method thread -s > $O/x3f_split2h.log 2>&1
echo "x3f exit $?" >> $O/x3f_split2h.log
grep -q "Fatal\|core dumped\|Segmentation" $O/x3f_split2h.log && exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_drq.py -q -rf --timeout 200 --timeout-method thread -s > $O/drq_tests.log 2>&1
echo "drq exit $?" >> $O/drq_tests.log
grep -q "Fatal\|core dumped\|Segmentation" $O/drq_tests.log && exit 1
timeout -k 10 300 python bench.py --workload atari_drq --no-cpu-baseline > $O/bench_drq_mfma.json 2> $O/bench_drq_mfma.err || exit 1
MTSAC_DRQ_MFMA=0 timeout -k 10 300 python bench.py --workload atari_drq --no-cpu-baseline > $O/bench_drq_valu.json 2> $O/bench_drq_valu.err || exit 1
bash tools/drq_kprof.sh r4c/drq_kprof_mfma > /dev/null 2>&1 || exit 1
MTSAC_DRQ_MFMA=0 bash tools/drq_kprof.sh r4c/drq_kprof_valu > /dev/null 2>&1 || exit 1
echo done
