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

typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));

// Where one 32x32 accumulator tile goes: pointers already offset to the batch entry.
struct TileOut {
  float* C;             // fp32 output or null
  long long ldc;
  const float* bias;    // EPI_BIAS_RELU
  const float* mask;    // EPI_RELU_MASK
  long long ldm;
  __bf16* Cp;           // split planes of the output or null
  long long ldcp, pC;
  int M, N;
  bool vec;             // every row start 16-B aligned (N, ldc, ldm, ldcp multiples of 4)
  // split2h (h2): the accumulator times unscale = 2^-(eA + eB); output planes are two fp16 planes
  // of x * oscale; the fp32 ReLU mask is read as is (x3p never takes a plane mask)
  bool h2;
  float unscale, oscale;
};

// ---- precision split2h: x * 2^e = h + l as two fp16 values (h = fp16(x 2^e), l = fp16(x 2^e - h);
// the subtraction is exact), with e per tensor chosen from an upper bound of |x| so that |x 2^e| <
// 2^15 (no overflow).  Elements above 2^-3 of the scaled range carry 22 significant bits; below,
// the absolute error is <= 2^-25 of the scaled unit.  A positive x whose planes would both round to
// zero keeps the smallest fp16 subnormal in l, so 'x > 0 <=> h > 0 or l > 0' holds exactly (the
// ReLU mask of the data grad reads the planes).
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// ---- the fragment layout of a B plane [rows][ldk] (ldk % 32 == 0, rows padded to 16): element
// (n, k) of fragment (n / 16, k / 32) -- 512 elements, 1 KB, contiguous in (n / 16, k / 32) order --
// at lane (n % 16) + 16 ((k / 8) % 4), element k % 8: the lane order of a v_mfma_*_16x16x32 B
// operand, so one wave load of a fragment reads 8 whole lines (row-major planes: 16 half lines)
__host__ __device__ inline long long frag_off(long long n, long long k, long long ldk) {
  return (((n >> 4) * (ldk >> 5) + (k >> 5)) << 9) + (((n & 15) + 16 * ((k >> 3) & 3)) << 3) + (k & 7);
}
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

__device__ inline void split2h_dev(float x, float s, _Float16& h, _Float16& l) {
  const float y = x * s;
  h = (_Float16)y;
  l = (_Float16)(y - (float)h);
  if (x > 0.f && h == (_Float16)0.f && l == (_Float16)0.f) l = __builtin_bit_cast(_Float16, (unsigned short)1);
}

// the planes' exponent for an upper bound of |x|: |x| 2^e < 2^15 (a margin of 2^-8 covers the fp32
// rounding of the bounded sums)
__device__ inline int plane_exp(float bound) {
  bound *= 1.00390625f;
  if (!(bound > 0.f) || !(bound < 3.0e38f)) return 0;
  int ex;
  (void)frexpf(bound, &ex);  // bound < 2^ex
  return min(100, max(-100, 15 - ex));
}

// block-wide max of one value per thread (every thread gets the result); scratch: 16 floats
__device__ inline float block_max_val(float m, float* scratch) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) scratch[threadIdx.x >> 6] = m;
  __syncthreads();
  float r = 0.f;
  for (int w = 0; w < (int)(blockDim.x + 63) / 64; ++w) r = fmaxf(r, scratch[w]);
  __syncthreads();
  return r;
}

// max over n recorded partial maxima, by the whole block (every thread gets the result); scratch: 16 floats
__device__ inline float block_max_of(const float* __restrict__ v, int n, float* scratch) {
  float m = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) m = fmaxf(m, v[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  __syncthreads();
  if ((threadIdx.x & 63) == 0) scratch[threadIdx.x >> 6] = m;
  __syncthreads();
  float r = 0.f;
  for (int w = 0; w < (int)(blockDim.x + 63) / 64; ++w) r = fmaxf(r, scratch[w]);
  __syncthreads();
  return r;
}

__device__ inline float exp2i(int e) { return __builtin_bit_cast(float, (unsigned)(127 + e) << 23); }  // |e| <= 126

// max |x| of a record's tensor: its partial maxima, or (none recorded) the planes' range 2^(15 - e)
__device__ inline float rec_max(const PlaneRec* r, int n, float* scratch) {
  if (r == nullptr) return 0.f;
  if (n <= 0) return exp2i(15 - r->e);
  return block_max_of(r->amax, n, scratch);
}

// the output planes' exponent of a split2h GEMM launch (SplitGemmParams bound inputs)
__device__ inline int gemm_out_exp(const SplitGemmParams& p, float* scratch) {
  const float ma = rec_max(p.ra, p.na, scratch);
  const float mb = rec_max(p.rb, p.nb, scratch);
  return plane_exp(p.kmul * ma * mb + (p.bias_in_b ? mb : 0.f));
}

__device__ inline void split3_dev(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)x;
  const float r1 = x - (float)h;
  m = (__bf16)r1;
  l = (__bf16)(r1 - (float)m);
}

// Epilogue of one 32x32 MFMA accumulator (col = lane & 31, row = (r&3) + 8(r>>2) + 4(lane>>5))
// at (row0, col0): restaged through a wave-private 32 x 36-float LDS scratch so every lane
// stores 16 B of fp32 (and 8 B of each bf16 plane) -- whole 128-B row segments per 8 lanes.
template <int EPI>
__device__ inline void store_tile32(const f32x16_t& acc, float* scr, int lane, int row0, int col0, const TileOut& o,
                                    float& omx) {
  const int lr = lane & 31, lh = lane >> 5;
#pragma unroll
  for (int r = 0; r < 16; ++r) scr[((r & 3) + 8 * (r >> 2) + 4 * lh) * 36 + lr] = acc[r];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int c4 = 4 * (lane & 7);
  const int col = col0 + c4;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int rr = (lane >> 3) + 8 * q;
    const int row = row0 + rr;
    if (row >= o.M) continue;
    float4 v = *reinterpret_cast<const float4*>(scr + rr * 36 + c4);
    float e[4] = {v.x, v.y, v.z, v.w};
    if (o.h2) {
#pragma unroll
      for (int j = 0; j < 4; ++j) e[j] *= o.unscale;
    }
    if (o.vec && col + 3 < o.N) {
      if (EPI == EPI_BIAS_RELU) {
        const float4 b = *reinterpret_cast<const float4*>(o.bias + col);
        e[0] = fmaxf(e[0] + b.x, 0.f); e[1] = fmaxf(e[1] + b.y, 0.f);
        e[2] = fmaxf(e[2] + b.z, 0.f); e[3] = fmaxf(e[3] + b.w, 0.f);
      }
      if (EPI == EPI_RELU_MASK) {
        const float4 mk = *reinterpret_cast<const float4*>(o.mask + (long long)row * o.ldm + col);
        e[0] = mk.x > 0.f ? e[0] : 0.f; e[1] = mk.y > 0.f ? e[1] : 0.f;
        e[2] = mk.z > 0.f ? e[2] : 0.f; e[3] = mk.w > 0.f ? e[3] : 0.f;
      }
      if (o.C) *reinterpret_cast<float4*>(o.C + (long long)row * o.ldc + col) = make_float4(e[0], e[1], e[2], e[3]);
      if (o.Cp && o.h2) {
        f16x4 h, l;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          _Float16 a, b;
          split2h_dev(e[j], o.oscale, a, b);
          h[j] = a; l[j] = b;
          omx = fmaxf(omx, fabsf(e[j]));
        }
        __bf16* cp = o.Cp + (long long)row * o.ldcp + col;
        *reinterpret_cast<f16x4*>(cp) = h;
        *reinterpret_cast<f16x4*>(cp + o.pC) = l;
      } else if (o.Cp) {
        bf16x4_t h, m, l;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          __bf16 a, b, c;
          split3_dev(e[j], a, b, c);
          h[j] = a; m[j] = b; l[j] = c;
        }
        __bf16* cp = o.Cp + (long long)row * o.ldcp + col;
        *reinterpret_cast<bf16x4_t*>(cp) = h;
        *reinterpret_cast<bf16x4_t*>(cp + o.pC) = m;
        *reinterpret_cast<bf16x4_t*>(cp + 2 * o.pC) = l;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int cc = col + j;
        if (cc >= o.N) continue;
        float x = e[j];
        if (EPI == EPI_BIAS_RELU) x = fmaxf(x + o.bias[cc], 0.f);
        if (EPI == EPI_RELU_MASK) x = o.mask[(long long)row * o.ldm + cc] > 0.f ? x : 0.f;
        if (o.C) o.C[(long long)row * o.ldc + cc] = x;
        if (o.Cp && o.h2) {
          _Float16 a, b;
          split2h_dev(x, o.oscale, a, b);
          omx = fmaxf(omx, fabsf(x));
          reinterpret_cast<_Float16*>(o.Cp)[(long long)row * o.ldcp + cc] = a;
          reinterpret_cast<_Float16*>(o.Cp)[(long long)row * o.ldcp + cc + o.pC] = b;
        } else if (o.Cp) {
          __bf16 a, b, c;
          split3_dev(x, a, b, c);
          __bf16* cp = o.Cp + (long long)row * o.ldcp + cc;
          cp[0] = a;
          cp[o.pC] = b;
          cp[2 * o.pC] = c;
        }
      }
    }
  }
  // the next tile's scratch writes must not pass this tile's reads (LDS is in order per wave)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace mtsac
