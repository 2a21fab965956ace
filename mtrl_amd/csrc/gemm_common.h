// gemm_common.h -- device-side operand addressing shared by the fp32 and split GEMM kernels.
#pragma once
#include "kernels.h"

namespace mtsac {

// The (batch entry, K slice) a workgroup works on: operand bases moved to the slice's first k,
// and the output (C or the split-K partial slab) it writes.
struct GemmSlice {
  const float* A;
  const float* B;
  float* C;
  float* db;
  int K, ldc, z;
};

template <bool TA, bool TB>
__device__ inline GemmSlice gemm_slice(const GemmParams& p) {
  GemmSlice s;
  const int S = p.splits > 1 ? p.splits : 1;
  const int zz = blockIdx.z, z = zz / S, sp = zz - z * S;
  const int k0 = sp * p.kchunk;
  s.z = z;
  s.K = S > 1 ? min(p.kchunk, p.K - k0) : p.K;
  s.A = p.A + z * p.sA + (TA ? (long long)k0 * p.lda : (long long)k0);
  s.B = p.B + z * p.sB + (TB ? (long long)k0 : (long long)k0 * p.ldb);
  if (S > 1) {
    const long long slab = (long long)p.M * p.N;
    s.C = p.ws + zz * slab;
    s.ldc = p.N;
    s.db = p.db ? p.ws + (long long)gridDim.z * slab + (long long)zz * p.N : nullptr;
  } else {
    s.C = p.C + z * p.sC;
    s.ldc = p.ldc;
    s.db = p.db ? p.db + z * p.sDb : nullptr;
  }
  return s;
}

}  // namespace mtsac
