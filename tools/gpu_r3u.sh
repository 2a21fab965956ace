# gpu_r3u.sh -- W400 whole-step flake vs hardware-queue sharing: 6 tries with GPU_MAX_HW_QUEUES=8,
# then 4 with the box default (4)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3u
mkdir -p $O
for q in 8 8 8 8 8 8 d d d d; do
  echo "== queues $q" >> $O/t.log
  if [ $q = d ]; then
    timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "buffer_async or conflict or drq or fullbatch" >> $O/t.log 2>&1
  else
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "buffer_async or conflict or drq or fullbatch" >> $O/t.log 2>&1
  fi
  echo "rc $?" >> $O/t.log
done
echo done
