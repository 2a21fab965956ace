# gpu_r3o.sh -- pipelined-vs-whole W400 determinism: x3p k-major slices 8 vs 5, repeated
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3o
mkdir -p $O
T="tests/test_gpu_fullbatch.py::test_pipelined_steps_equal_whole_steps"
for g in 8 8 4 4; do
  echo "== granules $g" >> $O/t.log
  MTSAC_X3P_KMAJOR_GRANULES=$g timeout -k 10 200 python -u -m pytest "$T" -q --timeout 150 --timeout-method thread >> $O/t.log 2>&1
  echo "rc $?" >> $O/t.log
done
echo done
