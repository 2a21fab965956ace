# gpu_r3t.sh -- does collecting the whole tests/ tree matter for the W400 pipelined-test flake?
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3t
mkdir -p $O
for i in 1 2 3; do
  echo "== full-collection try $i" >> $O/t.log
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "buffer_async or conflict or drq or fullbatch" >> $O/t.log 2>&1
  echo "rc $?" >> $O/t.log
done
echo done
