# gpu_r3b.sh -- DrQ conv-gradient fix + merged [s | s'] actor forward: diagnostics, parity, shard step
# times (E=1 path knob A/B), serialised kernel sums, DrQ bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 300 python -u tools/drq_diag.py 16 128 192 256 > $O/drq_diag.txt 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests/test_gpu_drq.py tests/test_gpu_update.py tests/test_gpu_fullbatch.py tests/test_gpu_shard.py tests/test_gpu_multiprocess.py -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/shard_step.py 50 25 13 7 > $O/shard_steps.txt 2>&1 || exit 1
MTSAC_E1_X3P=1 timeout -k 10 300 python tools/shard_step.py 25 13 7 > $O/shard_steps_e1x3p.txt 2>&1 || exit 1
bash tools/kprof.sh r3b/kprof 7 50 > $O/kprof.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload atari_drq --no-cpu-baseline > $O/bench_drq.json 2> $O/bench_drq.err || exit 1
echo done
