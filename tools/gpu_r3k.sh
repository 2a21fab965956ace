# gpu_r3k.sh -- shard steps after the x3s routing fix + DrQ kernel profile
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullbatch.py tests/test_gpu_x3f.py tests/test_gpu_drq.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python tools/shard_step.py 50 13 7 > $O/shard_steps.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/kt_t7 -o run -- python $GRAFT_REPO_ROOT/tools/shard_prof.py 7 > $GRAFT_REPO_ROOT/$O/kt_t7.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python tools/kernel_sums.py $O/kt_t7/run_kernel_trace.csv 60 > $O/sums_t7.txt || exit 1
rm -rf $O/kt_t7
bash tools/drq_kprof.sh r3k/drq || exit 1
timeout -k 10 300 python bench.py --workload atari_drq --no-cpu-baseline > $O/bench_drq.json 2> $O/bench_drq.err || exit 1
echo done
