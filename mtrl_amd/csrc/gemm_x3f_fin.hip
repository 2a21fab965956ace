// gemm_x3f_fin.hip -- the split-K gemm_x3f instances with the in-launch finish (FIN, see
// gemm_x3f_impl.h): task-shard trunk GEMMs whose row tiles do not fill the chip, one launch instead
// of the raw-slab GEMM plus splitk_epilogue_kernel (and, for data grads, plus a column-sum pass).
// Opt-in (MTSAC_SPLITK_FIN=1): measured slower than the separate finishing pass on the task shards
// (profiles/r3t_fin_bench.txt; split2h pair hand-off: profiles/r5m_*).
#include "gemm_x3f_impl.h"

namespace mtsac {
namespace x3fk {

template <int BM, int NP>
static bool fin_at(const SplitGemmParams& q, int epi, dim3 grid, hipStream_t st) {
  const dim3 blk(512);
  const bool c = q.C != nullptr, pl = q.Cp != nullptr;
  if (epi == EPI_BIAS_RELU) {
    if (c && pl) hipLaunchKernelGGL((gemm_x3f_kernel<BM, EPI_BIAS_RELU, true, true, false, 0, NP, 8, true>), grid, blk, 0, st, q);
    else if (c) hipLaunchKernelGGL((gemm_x3f_kernel<BM, EPI_BIAS_RELU, true, false, false, 0, NP, 8, true>), grid, blk, 0, st, q);
    else if (pl) hipLaunchKernelGGL((gemm_x3f_kernel<BM, EPI_BIAS_RELU, false, true, false, 0, NP, 8, true>), grid, blk, 0, st, q);
    else return false;
    return true;
  }
  if (epi == EPI_RELU_MASK && q.mask16) {
    if (c && pl) hipLaunchKernelGGL((gemm_x3f_kernel<BM, EPI_RELU_MASK, true, true, true, 0, NP, 8, true>), grid, blk, 0, st, q);
    else if (pl) hipLaunchKernelGGL((gemm_x3f_kernel<BM, EPI_RELU_MASK, false, true, true, 0, NP, 8, true>), grid, blk, 0, st, q);
    else hipLaunchKernelGGL((gemm_x3f_kernel<BM, EPI_RELU_MASK, true, false, true, 0, NP, 8, true>), grid, blk, 0, st, q);
    return true;
  }
  return false;
}

}  // namespace x3fk

// Launches the FIN form when an instance exists for (bm, epilogue, outputs); false: the caller
// runs the raw-slab launch + finishing pass instead.
bool gemm_x3f_fin_supported(const SplitGemmParams& q, int epi, int bm) {
  if (q.cnt == nullptr || q.np == 1 || (bm != 128 && bm != 208)) return false;
  const bool c = q.C != nullptr, pl = q.Cp != nullptr;
  if (epi == EPI_BIAS_RELU) return c || pl;
  return epi == EPI_RELU_MASK && q.mask16 != nullptr && (c || pl);
}

bool gemm_x3f_fin(const SplitGemmParams& q, int epi, int bm, dim3 grid, hipStream_t st) {
  if (!gemm_x3f_fin_supported(q, epi, bm)) return false;
  if (q.np == 2)  // split2h: two slices only (the pair hand-off)
    return bm == 128 ? x3fk::fin_at<128, 2>(q, epi, grid, st) : x3fk::fin_at<208, 2>(q, epi, grid, st);
  return bm == 128 ? x3fk::fin_at<128, 3>(q, epi, grid, st) : x3fk::fin_at<208, 3>(q, epi, grid, st);
}

}  // namespace mtsac
