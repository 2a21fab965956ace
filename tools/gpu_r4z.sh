# gpu_r4z.sh -- round-4 final evidence, part 1: what the driver runs (pytest -m gpu, smoke, default
# bench with the CPU baseline, DrQ bench)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_check.sh r4z || exit 1
echo done
