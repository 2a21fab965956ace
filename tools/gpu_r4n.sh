# gpu_r4n.sh -- round-4: full GPU suite after the graph dependency fix; in-launch split-K finish A/B at
# S3 split2h; kernel stats of the default bench; split2h gemm_x3f ablations
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4n
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err || exit 1
MTSAC_SPLITK_FIN=1 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_fin.json 2> $O/bench_fin.err || exit 1
X3F_H2=1 X3F_ABL="0 2 3 64 131" timeout -k 10 200 python tools/x3f_ablate.py 20 > $O/x3f_ablate_h2.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/st -o run -- python $R/bench.py --no-cpu-baseline --steps 20 --warmup 2 --settle-s 1 > $R/$O/st.log 2>&1 || exit 1
cp $R/$O/st/run_kernel_stats.csv $R/$O/kernel_stats.csv
rm -rf $R/$O/st
echo done
