# gpu_r4o.sh -- round-4: weight planes in the fragment layout (gemm_x3f B wave loads read whole lines):
# full GPU suite, S3 bench with and without it, split2h forward microbench both layouts, kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4o
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest tests/test_gpu_x3f.py -q -rf -x --timeout 120 --timeout-method thread -k fragment > $O/tests_frag.log 2>&1 || exit 1
X3F_H2=1 X3F_ABL="0 64" timeout -k 10 200 python tools/x3f_ablate.py 20 > $O/x3f_h2_rowmajor.txt 2>&1 || exit 1
X3F_H2=1 X3F_FRAG=1 X3F_ABL="0 2" timeout -k 10 200 python tools/x3f_ablate.py 20 > $O/x3f_h2_frag.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_frag.json 2> $O/bench_frag.err || exit 1
MTSAC_BFRAG=0 timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_rowmajor.json 2> $O/bench_rowmajor.err || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/st -o run -- python $R/bench.py --no-cpu-baseline --steps 20 --warmup 2 --settle-s 1 > $R/$O/st.log 2>&1 || exit 1
cp $R/$O/st/run_kernel_stats.csv $R/$O/kernel_stats.csv
rm -rf $R/$O/st
echo done
