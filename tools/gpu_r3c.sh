set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3c
mkdir -p $O
timeout -k 10 300 python -u tools/drq_diag.py 16 64 128 192 256 > $O/drq_diag.txt 2>&1 || exit 1
echo done
