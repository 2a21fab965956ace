# gpu_r4h.sh -- round-4: x3f tile order (column tiles vs row tiles fastest inside an XCD's run) on the
# split2h probe shapes and the S3 bench; step_finish after the parallel weight-max reduction
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4h
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_update.py tests/test_gpu_fullbatch.py -q -rf -x -k "split2h or p3 or test_update" --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/h2_probe.py > $O/h2_probe_order0.txt 2>&1 || exit 1
MTSAC_X3F_ORDER=1 timeout -k 10 200 python -u tools/h2_probe.py > $O/h2_probe_order1.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_order0.json 2> $O/bench_order0.err || exit 1
MTSAC_X3F_ORDER=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_order1.json 2> $O/bench_order1.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/st -o run -- python $R/bench.py --no-cpu-baseline --steps 20 --warmup 2 --settle-s 1 > $R/$O/st.log 2>&1 || exit 1
cp $R/$O/st/run_kernel_stats.csv $R/$O/kernel_stats.csv
rm -rf $R/$O/st
echo done
