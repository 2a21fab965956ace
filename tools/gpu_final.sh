# gpu_final.sh TAG -- round-end evidence: what the driver runs (pytest -m gpu, smoke, default bench,
# DrQ bench) and the profiles behind the bench line (rocprofv3 kernel stats; PMC FETCH/WRITE passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-final}
bash tools/gpu_check.sh $TAG || exit 1
bash tools/profile_round.sh ${TAG}_prof || exit 1
echo final done
