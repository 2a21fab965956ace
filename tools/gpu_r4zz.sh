# gpu_r4zz.sh -- round-4 final check on the final tree: pytest -m gpu, smoke, default bench (CPU
# baseline), DrQ bench
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_check.sh r4zz || exit 1
echo done
