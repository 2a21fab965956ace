# frag_pmc.sh TAG -- PMC evidence for the weight-plane fragment layout: the S3 split2h hidden forward
# (gemm_x3f, E = 2, 6400 x 2048 x 2048, bias+ReLU, planes out) with row-major and fragment-layout B
# planes, every counter group of tools/gemm_pmc.sh; summaries to gpurun_out/TAG_{rowmajor,frag}/
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-frag_pmc}
bash tools/gemm_pmc.sh ${TAG}_rowmajor 1 $((1 | 256 | 8192)) 2 6400 2048 2048 10 || exit 1
bash tools/gemm_pmc.sh ${TAG}_frag 1 $((1 | 256 | 8192 | 16384)) 2 6400 2048 2048 10 || exit 1
echo done
