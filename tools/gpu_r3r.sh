# gpu_r3r.sh -- round-3 evidence (tests, smoke, benches, rocprof stats, PMC) + the shard timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_final.sh r3final || exit 1
O=gpurun_out/r3final
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/kt_tl -o run -- python $GRAFT_REPO_ROOT/tools/shard_timeline.py > $GRAFT_REPO_ROOT/$O/tl.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
python tools/step_timeline.py $O/kt_tl/run_kernel_trace.csv full > $O/shard7_timeline.txt || exit 1
rm -rf $O/kt_tl
timeout -k 10 300 python bench.py --workload mt10_w400 --no-cpu-baseline > $O/bench_c1.json 2> $O/bench_c1.err || exit 1
echo all done
