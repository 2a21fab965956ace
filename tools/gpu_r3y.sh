# gpu_r3y.sh -- round-3 evidence with one compute stream by default: tests, smoke, benches, rocprof
# stats + PMC, shard steps, the 1-rank RCCL shard timeline, C1 / C2-bf16 / S3-bf16 / DrQ lines
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_final.sh r3y || exit 1
O=gpurun_out/r3y
timeout -k 10 300 python tools/shard_step.py 50 25 13 7 > $O/shard_steps.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/kt_tl -o run -- python $GRAFT_REPO_ROOT/tools/shard_timeline.py > $GRAFT_REPO_ROOT/$O/tl.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python tools/step_timeline.py $O/kt_tl/run_kernel_trace.csv full > $O/shard7_timeline.txt || exit 1
rm -rf $O/kt_tl
timeout -k 10 300 python bench.py --workload mt10_w400 --no-cpu-baseline > $O/bench_c1.json 2> $O/bench_c1.err || exit 1
timeout -k 10 300 python bench.py --workload mt10_w2048 --precision bf16 --no-cpu-baseline > $O/bench_c2_bf16.json 2> $O/bench_c2_bf16.err || exit 1
timeout -k 10 300 python bench.py --workload mt10_w2048 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || exit 1
timeout -k 10 300 python bench.py --precision bf16 --no-cpu-baseline > $O/bench_s3_bf16.json 2> $O/bench_s3_bf16.err || exit 1
timeout -k 10 300 python bench.py --workload mt50_w400 --no-cpu-baseline > $O/bench_s4.json 2> $O/bench_s4.err || exit 1
echo all done
