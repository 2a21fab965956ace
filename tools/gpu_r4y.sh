# gpu_r4y.sh -- round-4: the twin critic head's dot products in one pass: head forms bitwise, full GPU
# suite, S3 bench, serialised S3 sums
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4y
mkdir -p $O
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullbatch.py -q -rf -x -s -k head_kernel_forms --timeout 500 --timeout-method thread > $O/tests_forms.log 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/$O/kt -o run -- python $R/tools/shard_prof.py 50 50 2048 3 > $R/$O/kt.log 2>&1 || exit 1
python $R/tools/kernel_sums.py $R/$O/kt/run_kernel_trace.csv 45 > $R/$O/sums_s3_split2h.txt || exit 1
rm -rf $R/$O/kt
echo done
