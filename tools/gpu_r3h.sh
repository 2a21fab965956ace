# gpu_r3h.sh -- narrow trunks: fp32-operand MFMA path vs split3 at W=400 (C1, S4)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3h
mkdir -p $O
for w in mt10_w400 mt50_w400; do
  for p in fp32 split3; do
    timeout -k 10 300 python bench.py --workload $w --precision $p --no-cpu-baseline > $O/bench_${w}_$p.json 2> $O/bench_${w}_$p.err || exit 1
  done
done
echo done
