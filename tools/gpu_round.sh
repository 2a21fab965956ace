# GPU round: tests, bench (both precisions), rocprof kernel stats of the default bench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -rf > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
for prec in split3 fp32; do
  timeout -k 10 400 python bench.py --steps 20 --warmup 3 --precision $prec ${BENCH_EXTRA} > gpurun_out/bench_$prec.json 2> gpurun_out/bench_$prec.err
  rc=$?; echo "bench exit $rc" >> gpurun_out/bench_$prec.err
  if [ $rc -ne 0 ]; then exit $rc; fi
done
if [ -n "$PROFILE" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --exec eager > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
  echo "rocprof exit $?" >> $GRAFT_REPO_ROOT/gpurun_out/prof.log
fi
