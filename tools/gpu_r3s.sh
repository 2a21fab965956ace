# gpu_r3s.sh -- race hunt after memory churn
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3s
mkdir -p $O
timeout -k 10 400 python tools/pipe_stress2.py 6 > $O/stress2.txt 2>&1 || exit 1
echo done
