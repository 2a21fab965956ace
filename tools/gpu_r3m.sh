# gpu_r3m.sh -- finish-kernel sums, W400 x3p wgrad sweep, bf16 split-K A/B at C2
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3m
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullbatch.py tests/test_gpu_update.py tests/test_gpu_x3f.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/x3p_w400.py > $O/x3p_w400.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload mt10_w2048 --precision bf16 --no-cpu-baseline > $O/bench_c2bf16.json 2> $O/bench_c2bf16.err || exit 1
MTSAC_BF16_SPLIT=1 timeout -k 10 300 python bench.py --workload mt10_w2048 --precision bf16 --no-cpu-baseline > $O/bench_c2bf16_split.json 2> $O/bench_c2bf16_split.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/kt_s3 -o run -- python $GRAFT_REPO_ROOT/tools/shard_prof.py 50 50 2048 1 > $GRAFT_REPO_ROOT/$O/kt_s3.log 2>&1 || exit 1
python $GRAFT_REPO_ROOT/tools/kernel_sums.py $GRAFT_REPO_ROOT/$O/kt_s3/run_kernel_trace.csv 60 > $GRAFT_REPO_ROOT/$O/sums_s3.txt || exit 1
rm -rf $GRAFT_REPO_ROOT/$O/kt_s3
echo done
