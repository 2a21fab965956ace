# c1_prof_ab.sh TAG -- tools/c1_prof.sh timelines of the default library (TAG_new) and of
# mtrl_amd/libmtsac_ab.so (TAG_old, stamp check waived), one after the other
set -o pipefail
bash tools/c1_prof.sh ${1}_new || exit 1
MTSAC_ALLOW_STALE_LIB=1 MTSAC_LIB=$GRAFT_REPO_ROOT/mtrl_amd/libmtsac_ab.so bash tools/c1_prof.sh ${1}_old || exit 1
echo done
