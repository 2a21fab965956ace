# gpu_r4v.sh -- round-4: which head-kernel rows-per-wave form changes the bits
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4v
mkdir -p $O
timeout -k 10 600 python -u tools/head_forms_probe.py > $O/head_forms.txt 2>&1 || exit 1
echo done
