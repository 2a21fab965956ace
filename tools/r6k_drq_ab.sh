# r6k_drq_ab.sh TAG: the DrQ GPU tests, the per-kernel conv sweep (row-tile vs legacy kernels, grid caps)
# and a same-box bench A/B (MTSAC_DRQ_LEGACY=7: the pre-round-6 conv kernels), alternating three times
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_drq.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/drq_conv_bench.py 20 --wg-sweep > $O/conv_bench.txt 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 --workload atari_drq > $O/new_$i.json 2>/dev/null || exit 1
  MTSAC_DRQ_LEGACY=7 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 --workload atari_drq > $O/old_$i.json 2>/dev/null || exit 1
done
echo benched
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/prof -o run -- python bench.py --workload atari_drq --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_bench.json 2>$O/prof.err || exit 1
python tools/rocpd_sums.py $O/prof/run_results.db drq_logs_kernel 45 > $O/kernel_sums.txt
echo profiled
