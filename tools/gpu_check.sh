# gpu_check.sh TAG -- what the driver runs at round end: pytest -m gpu, smoke(), default bench,
# plus the DrQ bench line; outputs under gpurun_out/TAG/.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-check}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python bench.py --workload atari_drq > $O/bench_drq.json 2> $O/bench_drq.err || exit 1
echo done
