# gpu_configs.sh TAG -- bench lines of the other BASELINE configs on the current tree
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-cfg}
mkdir -p $O
for w in mt10_w400 mt10_w2048 mt50_w400; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || exit 1
done
timeout -k 10 300 python bench.py --workload mt10_w2048 --precision split3 --no-cpu-baseline > $O/bench_mt10_w2048_split3.json 2> $O/bench_split3c2.err || exit 1
timeout -k 10 300 python bench.py --precision split3 --no-cpu-baseline > $O/bench_mt50_w2048_split3.json 2> $O/bench_split3s3.err || exit 1
timeout -k 10 300 python bench.py --workload mt10_w2048 --precision bf16 --no-cpu-baseline > $O/bench_mt10_w2048_bf16.json 2> $O/bench_bf16c2.err || exit 1
timeout -k 10 300 python bench.py --precision bf16 --no-cpu-baseline > $O/bench_mt50_w2048_bf16.json 2> $O/bench_bf16s3.err || exit 1
echo done
