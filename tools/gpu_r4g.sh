# gpu_r4g.sh -- round-4: the split2h 7-task shard's serialised kernel budget; input-layer weight grad
# on k-major planes vs on-the-fly at S3 under split2h
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4g
mkdir -p $O
R=$GRAFT_REPO_ROOT
MTSAC_INPUT_WGRAD=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_inwgrad_planes.json 2> $O/bench_inwgrad_planes.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$O/kt7 -o run -- python $R/tools/shard_prof.py 7 50 2048 3 > $R/$O/kt7.log 2>&1 || exit 1
python $R/tools/kernel_sums.py $R/$O/kt7/run_kernel_trace.csv 45 > $R/$O/sums_t7_split2h.txt || exit 1
rm -rf $R/$O/kt7
echo done
