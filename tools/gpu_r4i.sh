# gpu_r4i.sh -- round-4: the GPU suite on the current tree, default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4i
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --maxfail=10 --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/gpu_tests.log
grep -q "Fatal\|core dumped\|Segmentation" $O/gpu_tests.log && exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
echo done
