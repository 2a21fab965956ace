set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/it5
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_drq.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload atari_drq --cpu-steps 1 > $O/bench_x3.json 2> $O/bench_x3.err || exit 1
MTSAC_DRQ_GEMM=f32 timeout -k 10 300 python bench.py --workload atari_drq --cpu-steps 1 > $O/bench_f32.json 2> $O/bench_f32.err || exit 1
echo done
