# gpu_r3c.sh -- full GPU suite on the merged-actor tree, shard steps, serialised kernel sums, benches
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3c
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/shard_step.py 50 25 13 7 > $O/shard_steps.txt 2>&1 || exit 1
bash tools/kprof.sh r3c/kprof 7 50 > $O/kprof.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python bench.py --workload atari_drq --no-cpu-baseline > $O/bench_drq.json 2> $O/bench_drq.err || exit 1
echo done
