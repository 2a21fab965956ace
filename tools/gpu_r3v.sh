# gpu_r3v.sh -- lanes vs hardware queues: the W400 flake reproduction 4x (conftest raises the queues),
# the full GPU suite, C1 / S3 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3v
mkdir -p $O
for i in 1 2 3 4; do
  echo "== try $i" >> $O/t.log
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "buffer_async or conflict or drq or fullbatch" >> $O/t.log 2>&1
  echo "rc $?" >> $O/t.log
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --workload mt10_w400 --no-cpu-baseline > $O/bench_c1.json 2> $O/bench_c1.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_s3.json 2> $O/bench_s3.err || exit 1
timeout -k 10 300 python tools/shard_step.py 50 7 > $O/shard_steps.txt 2>&1 || exit 1
echo done
