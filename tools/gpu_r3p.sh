# gpu_r3p.sh -- pipelined / whole-step race hunt
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3p
mkdir -p $O
timeout -k 10 250 python tools/pipe_stress.py 10 10 400 1 8 > $O/w400.txt 2>&1 || exit 1
timeout -k 10 250 python tools/pipe_stress.py 50 7 2048 1 4 > $O/t7.txt 2>&1 || exit 1
timeout -k 10 250 python tools/pipe_stress.py 10 10 2048 2 4 > $O/c2bf16.txt 2>&1 || exit 1
echo done
