# gpu_r4j.sh -- round-4: the GPU suite on the current tree (two-block x3f epilogue, build stamp, split2h
# compat default), the probe, the S3 bench (split2h and split3), kernel stats of a short default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4j
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --maxfail=10 --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/gpu_tests.log
grep -q "Fatal\|core dumped\|Segmentation" $O/gpu_tests.log && exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/h2_probe.py > $O/h2_probe.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --precision split3 > $O/bench_split3.json 2> $O/bench_split3.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/st -o run -- python $R/bench.py --no-cpu-baseline --steps 20 --warmup 2 --settle-s 1 > $R/$O/st.log 2>&1 || exit 1
cp $R/$O/st/run_kernel_stats.csv $R/$O/kernel_stats.csv
rm -rf $R/$O/st
echo done
