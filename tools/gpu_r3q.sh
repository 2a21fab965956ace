# gpu_r3q.sh -- reproduce the r3n pipelined-test failure in the full-suite order (3 tries)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3q
mkdir -p $O
for i in 1 2 3; do
  echo "== try $i" >> $O/t.log
  timeout -k 10 300 python -u -m pytest tests/test_gpu_buffer_async.py tests/test_gpu_conflict.py tests/test_gpu_drq.py tests/test_gpu_fullbatch.py -m gpu -q -rf --timeout 200 --timeout-method thread >> $O/t.log 2>&1
  echo "rc $?" >> $O/t.log
done
echo done
