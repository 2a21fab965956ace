# gpu_r3w.sh -- lane mode by the start-time queue count: the flaky-subset 4x, the full GPU suite,
# C1 / S3 benches (respawned with 16 queues) and C1 at 4 queues (one stream) for the cost
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3w
mkdir -p $O
for i in 1 2 3 4; do
  echo "== try $i" >> $O/t.log
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "buffer_async or conflict or drq or fullbatch" >> $O/t.log 2>&1
  echo "rc $?" >> $O/t.log
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload mt10_w400 --no-cpu-baseline > $O/bench_c1.json 2> $O/bench_c1.err || exit 1
MTSAC_HWQ_CHILD=1 timeout -k 10 300 python bench.py --workload mt10_w400 --no-cpu-baseline > $O/bench_c1_onestream.json 2> $O/bench_c1_onestream.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_s3.json 2> $O/bench_s3.err || exit 1
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python tools/shard_step.py 50 13 7 > $O/shard_steps.txt 2>&1 || exit 1
echo done
