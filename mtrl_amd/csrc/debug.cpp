// debug.cpp -- test-only entry points (include/mtsac_debug.h) for the plane GEMM.
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/mtsac.h"
#include "../../include/mtsac_debug.h"
#include "kernels.h"

using namespace mtsac;

namespace {

long long up32(long long x) { return (x + 31) / 32 * 32; }

__global__ void fill_rand_f32(float* p, long long n, unsigned seed) {
  long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned x = (unsigned)i * 2654435761u ^ seed;
  x ^= x >> 13;
  x *= 0x5bd1e995u;
  x ^= x >> 15;
  p[i] = ((float)(x & 0xFFFFFF) / 8388608.0f) - 1.0f;
}

struct DevBuf {
  std::vector<void*> ptrs;
  ~DevBuf() {
    for (void* p : ptrs) (void)hipFree(p);
  }
  template <typename T>
  T* get(size_t n) {
    void* p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) return nullptr;
    (void)hipMemset(p, 0, std::max<size_t>(n, 1) * sizeof(T));
    ptrs.push_back(p);
    return reinterpret_cast<T*>(p);
  }
};

// planes of an operand that the GEMM reads as [rows][K]; source fp32 either [rows][K] or [K][rows]
__bf16* make_planes(DevBuf& db, const float* dsrc, int rows, int K, bool kmajor, long long& ld, long long& ps) {
  ld = up32(K);
  ps = (long long)rows * ld;
  __bf16* out = db.get<__bf16>(3 * ps);
  if (!out) return nullptr;
  SplitParams s{};
  s.x = dsrc;
  s.ldx = kmajor ? rows : K;
  s.rows = kmajor ? K : rows;
  s.cols = kmajor ? rows : K;
  s.out = out;
  s.ldo = ld;
  s.po = ps;
  s.out_rows = rows;
  s.out_cols = (int)ld;
  split_planes(s, kmajor, 1, nullptr);
  return out;
}

}  // namespace

extern "C" {

int mtsac_debug_gemm_x3p(int epi, int M, int N, int K, const float* A, int a_kmajor, const float* B, int b_kmajor,
                         float* C, const float* bias, const float* mask) {
  if (M < 1 || N < 1 || K < 1 || !A || !B || !C) return -22;
  DevBuf d;
  float* dA = d.get<float>((size_t)M * K);
  float* dB = d.get<float>((size_t)N * K);
  float* dC = d.get<float>((size_t)M * N);
  float* dbias = d.get<float>(N);
  float* dmask = d.get<float>((size_t)M * N);
  if (!dA || !dB || !dC || !dbias || !dmask) return -12;
  (void)hipMemcpy(dA, A, sizeof(float) * M * K, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, B, sizeof(float) * N * K, hipMemcpyHostToDevice);
  if (bias) (void)hipMemcpy(dbias, bias, sizeof(float) * N, hipMemcpyHostToDevice);
  if (mask) (void)hipMemcpy(dmask, mask, sizeof(float) * M * N, hipMemcpyHostToDevice);
  long long lda, pa, ldb, pb;
  __bf16* Ap = make_planes(d, dA, M, K, a_kmajor != 0, lda, pa);
  __bf16* Bp = make_planes(d, dB, N, K, b_kmajor != 0, ldb, pb);
  if (!Ap || !Bp) return -12;
  SplitGemmParams g{};
  g.A = Ap;
  g.lda = lda;
  g.pA = pa;
  g.B = Bp;
  g.ldb = ldb;
  g.pB = pb;
  g.C = dC;
  g.ldc = N;
  g.bias = dbias;
  g.mask = dmask;
  g.ldm = N;
  g.M = M;
  g.N = N;
  g.K = (int)lda;
  gemm_x3p(g, epi, 1, nullptr);
  if (hipDeviceSynchronize() != hipSuccess) return -5;
  if (hipMemcpy(C, dC, sizeof(float) * M * N, hipMemcpyDeviceToHost) != hipSuccess) return -5;
  return 0;
}

int mtsac_debug_gemm_x3p_bench(int epi, int batch, int M, int N, int K, int iters, double* ms_per_launch) {
  if (M < 1 || N < 1 || K < 1 || batch < 1 || iters < 1 || !ms_per_launch) return -22;
  DevBuf d;
  const long long ld = up32(K);
  const long long pa = (long long)M * ld, pb = (long long)N * ld;
  float* fa = d.get<float>((size_t)M * K);
  float* fb = d.get<float>((size_t)N * K);
  __bf16* Ap = d.get<__bf16>((size_t)3 * pa * batch);
  __bf16* Bp = d.get<__bf16>((size_t)3 * pb * batch);
  float* C = d.get<float>((size_t)M * N * batch);
  float* bias = d.get<float>((size_t)N * batch);
  if (!fa || !fb || !Ap || !Bp || !C || !bias) return -12;
  hipLaunchKernelGGL(fill_rand_f32, dim3((unsigned)(((long long)M * K + 255) / 256)), dim3(256), 0, nullptr, fa,
                     (long long)M * K, 3u);
  hipLaunchKernelGGL(fill_rand_f32, dim3((unsigned)(((long long)N * K + 255) / 256)), dim3(256), 0, nullptr, fb,
                     (long long)N * K, 5u);
  for (int z = 0; z < batch; ++z) {
    SplitParams s{};
    s.x = fa; s.ldx = K; s.rows = M; s.cols = K; s.out = Ap + z * 3 * pa; s.ldo = ld; s.po = pa;
    s.out_rows = M; s.out_cols = (int)ld;
    split_planes(s, false, 1, nullptr);
    s.x = fb; s.rows = N; s.out = Bp + z * 3 * pb; s.po = pb; s.out_rows = N;
    split_planes(s, false, 1, nullptr);
  }
  SplitGemmParams g{};
  g.A = Ap; g.lda = ld; g.pA = pa; g.sA = 3 * pa;
  g.B = Bp; g.ldb = ld; g.pB = pb; g.sB = 3 * pb;
  g.C = C; g.ldc = N; g.sC = (long long)M * N;
  g.bias = bias; g.sBias = N;
  g.mask = C; g.ldm = N; g.sMask = (long long)M * N;
  g.M = M; g.N = N; g.K = (int)ld;
  gemm_x3p(g, epi, batch, nullptr);
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return -5;
  (void)hipEventRecord(e0, nullptr);
  for (int i = 0; i < iters; ++i) gemm_x3p(g, epi, batch, nullptr);
  (void)hipEventRecord(e1, nullptr);
  if (hipEventSynchronize(e1) != hipSuccess) return -5;
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  *ms_per_launch = ms / iters;
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return 0;
}

int mtsac_debug_x3p_geo(int geo) {
  const int old = g_x3p_geo;
  if ((geo & 255) <= 1) g_x3p_geo = geo & 255;
  g_x3p_dbg = geo >> 8;
  return old;
}

}  // extern "C"
