# gpu_r4f.sh -- round-4: the driver's checks on the split2h-default tree (pytest -m gpu, smoke, bench,
# DrQ bench), the profiles behind the bench line, the other configs' bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_check.sh r4f || exit 1
bash tools/profile_round.sh r4f_prof split2h || exit 1
bash tools/gpu_configs.sh r4f_cfg || exit 1
echo done
