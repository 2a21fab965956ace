# gpu_r3gg.sh -- input-wgrad form by batch size: full GPU suite, smoke, S3 / C1 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3gg
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python bench.py --workload mt10_w400 --no-cpu-baseline > $O/bench_c1.json 2> $O/bench_c1.err || exit 1
echo done
