// devrng.h -- device random streams of the engine.
//
// 1. pcg64_*: numpy's PCG64 (XSL-RR 128/64) arithmetic with the 128-bit LCG done in
//    64-bit halves; used by the replay index kernel to reproduce
//    np.random.default_rng(seed).integers bit for bit (buffers.py:260,523-527).
// 2. philox4x32-10 + Box-Muller: a counter-based N(0,1) stream for the policy noise
//    when no epsilon is injected (the reference uses JAX threefry, mtsac.py:355,629,
//    which is not reproduced; parity is defined given injected noise).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mtsac {

struct u128 {
  unsigned long long hi, lo;
};

__device__ __host__ inline u128 mul128(u128 a, u128 b) {
  u128 r;
  r.lo = a.lo * b.lo;
#if defined(__HIP_DEVICE_COMPILE__)
  unsigned long long h = __umul64hi(a.lo, b.lo);
#else
  unsigned long long h = (unsigned long long)(((unsigned __int128)a.lo * b.lo) >> 64);
#endif
  r.hi = h + a.lo * b.hi + a.hi * b.lo;
  return r;
}

__device__ __host__ inline u128 add128(u128 a, u128 b) {
  u128 r;
  r.lo = a.lo + b.lo;
  r.hi = a.hi + b.hi + (r.lo < a.lo ? 1ull : 0ull);
  return r;
}

// XSL-RR output of an (already stepped) state
__device__ __host__ inline unsigned long long pcg64_output(u128 s) {
  const unsigned long long x = s.hi ^ s.lo;
  const unsigned rot = (unsigned)(s.hi >> 58);
  return (x >> rot) | (x << ((64u - rot) & 63u));
}

// ---------------------------------------------------------------- philox4x32-10
__device__ inline void philox4x32_10(uint32_t ctr[4], uint32_t key0, uint32_t key1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(M0, ctr[0]), lo0 = M0 * ctr[0];
    const uint32_t hi1 = __umulhi(M1, ctr[2]), lo1 = M1 * ctr[2];
    const uint32_t n0 = hi1 ^ ctr[1] ^ key0;
    const uint32_t n2 = hi0 ^ ctr[3] ^ key1;
    ctr[0] = n0;
    ctr[1] = lo1;
    ctr[2] = n2;
    ctr[3] = lo0;
    key0 += W0;
    key1 += W1;
  }
}

__device__ inline float u32_to_unit_open(uint32_t x) {  // (0, 1]
  return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f);
}

// four N(0,1) variates for (seed, stream, counter, row)
__device__ inline void normal4(unsigned long long seed, uint32_t stream, unsigned long long counter, uint32_t row,
                               float out[4]) {
  uint32_t c[4] = {row, stream, (uint32_t)counter, (uint32_t)(counter >> 32)};
  philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  const float u1 = u32_to_unit_open(c[0]), u2 = u32_to_unit_open(c[1]);
  const float u3 = u32_to_unit_open(c[2]), u4 = u32_to_unit_open(c[3]);
  const float r1 = sqrtf(-2.0f * logf(u1)), r2 = sqrtf(-2.0f * logf(u3));
  const float t1 = 6.28318530717958647692f * u2, t2 = 6.28318530717958647692f * u4;
  out[0] = r1 * cosf(t1);
  out[1] = r1 * sinf(t1);
  out[2] = r2 * cosf(t2);
  out[3] = r2 * sinf(t2);
}

__device__ inline void uniform4(unsigned long long seed, uint32_t stream, unsigned long long counter, uint32_t row,
                                float out[4]) {
  uint32_t c[4] = {row, stream, (uint32_t)counter, (uint32_t)(counter >> 32)};
  philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
  for (int i = 0; i < 4; ++i) out[i] = (float)(c[i] >> 8) * (1.0f / 16777216.0f);  // [0,1)
}

}  // namespace mtsac
