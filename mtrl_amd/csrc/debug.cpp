// debug.cpp -- test-only entry points (include/mtsac_debug.h) for the plane GEMM.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mtsac.h"
#include "../../include/mtsac_debug.h"
#include "drq_kernels.h"
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

long long up8(long long x) { return (x + 7) / 8 * 8; }

// planes of a fp32 operand stored [rows][K] (k contiguous) or, kmajor, [K][rows]; split in its
// stored orientation: row-major planes [3][rows][up32(K)], k-major planes [3][up32(K)][up8(rows)]
// (zeros in the padding)
void plane_geom(int rows, int K, bool kmajor, long long& ld, long long& ps) {
  ld = kmajor ? up8(rows) : up32(K);
  ps = (kmajor ? up32(K) : (long long)rows) * ld;
}

void split_into(const float* dsrc, int rows, int K, bool kmajor, __bf16* out, const int* e2h = nullptr,
                bool frag = false) {
  long long ld, ps;
  plane_geom(rows, K, kmajor, ld, ps);
  SplitParams s{};
  s.x = dsrc;
  s.ldx = kmajor ? rows : K;
  s.rows = kmajor ? K : rows;
  s.cols = kmajor ? rows : K;
  s.out_rows = kmajor ? (int)up32(K) : rows;
  s.out = out;
  s.ldo = ld;
  s.po = ps;
  s.out_cols = (int)ld;
  s.e2h = e2h;
  s.frag = frag ? 1 : 0;
  split_planes(s, false, 1, nullptr);
}

__bf16* make_planes(DevBuf& db, const float* dsrc, int rows, int K, bool kmajor, long long& ld, long long& ps) {
  plane_geom(rows, K, kmajor, ld, ps);
  __bf16* out = db.get<__bf16>(3 * ps);
  if (out) split_into(dsrc, rows, K, kmajor, out);
  return out;
}

}  // namespace

extern "C" {

int mtsac_debug_gemm_x3p(int epi, int M, int N, int K, const float* A, int a_kmajor, const float* B, int b_kmajor,
                         float* C, const float* bias, const float* mask, float* Csum) {
  const int splits = (epi >> 8) & 255;
  epi &= 255;
  if (M < 1 || N < 1 || K < 1 || !A || !B || !C) return -22;
  DevBuf d;
  float* dA = d.get<float>((size_t)M * K);
  float* dB = d.get<float>((size_t)N * K);
  float* dC = d.get<float>((size_t)M * N);
  float* dbias = d.get<float>(N);
  float* dmask = d.get<float>((size_t)M * N);
  __bf16* dCp = d.get<__bf16>((size_t)3 * M * N);
  float* dws = d.get<float>(splits > 1 ? (size_t)gemm_ws_floats(M, N, 1, splits) : 1);
  if (!dA || !dB || !dC || !dbias || !dmask || !dCp || !dws) return -12;
  (void)hipMemcpy(dA, A, sizeof(float) * M * K, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, B, sizeof(float) * N * K, hipMemcpyHostToDevice);
  if (bias) (void)hipMemcpy(dbias, bias, sizeof(float) * N, hipMemcpyHostToDevice);
  if (mask) (void)hipMemcpy(dmask, mask, sizeof(float) * M * N, hipMemcpyHostToDevice);
  long long lda, pa, ldb, pb;
  __bf16* Ap = make_planes(d, dA, M, K, a_kmajor != 0, lda, pa);
  __bf16* Bp = make_planes(d, dB, N, K, b_kmajor != 0, ldb, pb);
  if (!Ap || !Bp) return -12;
  SplitGemmParams g{};
  g.A = Ap; g.lda = lda; g.pA = pa; g.a_kmajor = a_kmajor != 0;
  g.B = Bp; g.ldb = ldb; g.pB = pb; g.b_kmajor = b_kmajor != 0;
  g.C = dC; g.ldc = N;
  g.bias = dbias;
  g.mask = dmask; g.ldm = N;
  if (Csum) {
    g.Cp = dCp; g.ldcp = N; g.pC = (long long)M * N;
  }
  g.M = M; g.N = N; g.K = (int)up32(K);
  g.splits = splits;
  g.ws = dws;
  gemm_x3p(g, epi, 1, nullptr);
  if (hipDeviceSynchronize() != hipSuccess) return -5;
  if (hipMemcpy(C, dC, sizeof(float) * M * N, hipMemcpyDeviceToHost) != hipSuccess) return -5;
  if (Csum) {
    std::vector<__bf16> h((size_t)3 * M * N);
    if (hipMemcpy(h.data(), dCp, sizeof(__bf16) * h.size(), hipMemcpyDeviceToHost) != hipSuccess) return -5;
    const size_t n = (size_t)M * N;
    for (size_t i = 0; i < n; ++i) Csum[i] = ((float)h[i] + (float)h[n + i]) + (float)h[2 * n + i];
  }
  return 0;
}

int mtsac_debug_gemm_x3p_bench(int epi, int batch, int M, int N, int K, int iters, double* ms_per_launch) {
  const int layout = (epi >> 8) & 3;  // bit 0: A k-major, bit 1: B k-major
  const int splits = (epi >> 16) & 255;  // split-K slices (0/1: none; EPI_STORE: + splitk_reduce; 255: auto)
  const bool fin = (epi >> 12) & 1;      // arrival counters: the weight grads' in-launch reduce
  const bool h2 = (epi >> 13) & 1;       // precision split2h (zero exponents: operands in [-1, 1])
  const bool pout = (epi >> 14) & 1;     // output planes too (the forward's: bias+ReLU planes out)
  epi &= 255;
  if (M < 1 || N < 1 || K < 1 || batch < 1 || iters < 1 || !ms_per_launch) return -22;
  DevBuf d;
  PlaneRec* rec = h2 ? d.get<PlaneRec>(3) : nullptr;
  float* fa = d.get<float>((size_t)M * K);
  float* fb = d.get<float>((size_t)N * K);
  float* C = d.get<float>((size_t)M * N * batch);
  float* bias = d.get<float>((size_t)N * batch);
  if (!fa || !fb || !C || !bias) return -12;
  hipLaunchKernelGGL(fill_rand_f32, dim3((unsigned)(((long long)M * K + 255) / 256)), dim3(256), 0, nullptr, fa,
                     (long long)M * K, 3u);
  hipLaunchKernelGGL(fill_rand_f32, dim3((unsigned)(((long long)N * K + 255) / 256)), dim3(256), 0, nullptr, fb,
                     (long long)N * K, 5u);
  // one plane set per batch entry (distinct memory, same values)
  long long lda, pa, ldb, pb;
  plane_geom(M, K, layout & 1, lda, pa);
  plane_geom(N, K, layout & 2, ldb, pb);
  __bf16* Ap = d.get<__bf16>((size_t)3 * pa * batch);
  __bf16* Bp = d.get<__bf16>((size_t)3 * pb * batch);
  if (!Ap || !Bp) return -12;
  for (int z = 0; z < batch; ++z) {
    split_into(fa, M, K, layout & 1, Ap + 3 * pa * z, h2 ? &rec[0].e : nullptr);
    split_into(fb, N, K, layout & 2, Bp + 3 * pb * z, h2 ? &rec[1].e : nullptr);
  }
  SplitGemmParams g{};
  if (h2) {
    g.np = 2;
    g.ra = rec; g.rb = rec + 1; g.rc = rec + 2;
    g.kmul = (float)K;
  }
  if (pout) {
    __bf16* Cp = d.get<__bf16>((size_t)3 * M * N * batch);
    if (!Cp) return -12;
    g.Cp = Cp; g.ldcp = N; g.pC = (long long)M * N; g.sCp = 3 * g.pC;
  }
  const bool planes_only = pout;
  g.A = Ap; g.lda = lda; g.pA = pa; g.sA = 3 * pa; g.a_kmajor = layout & 1;
  g.B = Bp; g.ldb = ldb; g.pB = pb; g.sB = 3 * pb; g.b_kmajor = (layout >> 1) & 1;
  g.C = planes_only ? nullptr : C; g.ldc = N; g.sC = (long long)M * N;
  g.bias = bias; g.sBias = N;
  g.mask = C; g.ldm = N; g.sMask = (long long)M * N;
  g.M = M; g.N = N; g.K = (int)up32(K);
  if (splits > 1) {
    g.splits = splits == 255 ? -1 : splits;
    const int sw = splits == 255 ? gemm_x3p_splits(M, N, g.K, batch, layout == 3) : splits;
    g.ws = d.get<float>((size_t)M * N * batch * std::max(sw, 1));
    if (!g.ws) return -12;
    if (fin) {
      g.cnt = d.get<int>((size_t)GEMM_X3F_CNT);
      if (!g.cnt) return -12;
    }
  }
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

// gemm_x3f (row-major x row-major planes, K % 64 == 0): C[M][N] = A[M][K] . B[N][K]^T from host
// fp32 arrays, epi 1 bias+ReLU / 2 ReLU mask (fp32 mask, or with bit 8 of epi its bf16 high
// plane); Csum (nullable) receives the sum of the written planes.  -95 when gemm_x3f does not take
// the shape (too few tiles, layout).
int mtsac_debug_gemm_x3f(int epi, int batch, int M, int N, int K, const float* A, const float* B, float* C,
                         const float* bias, const float* mask, float* Csum) {
  const bool m16 = (epi >> 8) & 1;
  const bool small = (epi >> 9) & 1;  // gemm_x3s instead
  const int np = ((epi >> 10) & 1) ? 1 : 3;  // bf16: the high plane only
  const bool autosplit = (epi >> 11) & 1;     // split-K by the launcher's own choice (workspace given)
  const bool fin = (epi >> 12) & 1;           // ... with arrival counters: the in-launch finish
  const bool h2 = (epi >> 13) & 1;            // precision split2h: fp16 planes scaled per tensor
  const bool bfrag = (epi >> 14) & 1;         // B planes in the fragment layout (N % 16 == 0)
  epi &= 255;
  if (M < 1 || N < 1 || K < 1 || batch < 1 || !A || !B || !C) return -22;
  if (bfrag && N % 16 != 0) return -22;
  DevBuf d;
  const size_t nA = (size_t)M * K * batch, nB = (size_t)N * K * batch, nC = (size_t)M * N * batch;
  // split2h: records of A, B (its max covering the bias, as a trunk record does), the mask and C
  PlaneRec* rec = d.get<PlaneRec>(4);
  if (!rec) return -12;
  if (h2) {
    auto amax = [](const float* x, size_t n) {
      float m = 0.f;
      for (size_t i = 0; i < n; ++i) m = std::max(m, std::fabs(x[i]));
      return m;
    };
    auto pexp = [](float b) {
      b *= 1.00390625f;
      if (!(b > 0.f)) return 0;
      int ex;
      (void)std::frexp(b, &ex);
      return 15 - ex;
    };
    const float ma = amax(A, nA), mbias = (epi == 1 && bias) ? amax(bias, (size_t)N * batch) : 0.f;
    const float mb = std::max(amax(B, nB), mbias);
    const float mm = mask ? amax(mask, nC) : 1.f;
    std::vector<PlaneRec> h(4);
    std::memset(h.data(), 0, sizeof(PlaneRec) * 4);
    h[0].e = pexp(ma); h[0].amax[0] = ma;
    h[1].e = pexp(mb); h[1].amax[0] = mb;
    h[2].e = pexp(mm); h[2].amax[0] = mm;
    (void)hipMemcpy(rec, h.data(), sizeof(PlaneRec) * 4, hipMemcpyHostToDevice);
  }
  float* dA = d.get<float>(nA);
  float* dB = d.get<float>(nB);
  float* dC = d.get<float>(nC);
  float* dbias = d.get<float>((size_t)N * batch);
  float* dmask = d.get<float>(nC);
  __bf16* dCp = d.get<__bf16>(3 * nC);
  __bf16* dM16 = d.get<__bf16>(3 * nC);
  if (!dA || !dB || !dC || !dbias || !dmask || !dCp || !dM16) return -12;
  (void)hipMemcpy(dA, A, sizeof(float) * nA, hipMemcpyHostToDevice);
  (void)hipMemcpy(dB, B, sizeof(float) * nB, hipMemcpyHostToDevice);
  if (bias) (void)hipMemcpy(dbias, bias, sizeof(float) * N * batch, hipMemcpyHostToDevice);
  if (mask) (void)hipMemcpy(dmask, mask, sizeof(float) * nC, hipMemcpyHostToDevice);
  const long long Kp = (K + 63) / 64 * 64;
  __bf16* Ap = d.get<__bf16>((size_t)3 * M * Kp * batch);
  __bf16* Bp = d.get<__bf16>((size_t)3 * N * Kp * batch);
  if (!Ap || !Bp) return -12;
  for (int z = 0; z < batch; ++z) {
    SplitParams s{};
    s.x = dA + (size_t)z * M * K; s.ldx = K; s.rows = M; s.cols = K;
    s.out = Ap + (size_t)z * 3 * M * Kp; s.ldo = Kp; s.po = (long long)M * Kp; s.out_rows = M; s.out_cols = (int)Kp;
    s.e2h = h2 ? &rec[0].e : nullptr;
    split_planes(s, false, 1, nullptr);
    s.x = dB + (size_t)z * N * K; s.rows = N;
    s.out = Bp + (size_t)z * 3 * N * Kp; s.po = (long long)N * Kp; s.out_rows = N;
    s.e2h = h2 ? &rec[1].e : nullptr;
    s.frag = bfrag ? 1 : 0;
    split_planes(s, false, 1, nullptr);
    s.frag = 0;
    if (m16) {  // planes of the mask, row stride N
      s.x = dmask + (size_t)z * M * N; s.ldx = N; s.rows = M; s.cols = N;
      s.out = dM16 + (size_t)z * 3 * M * N; s.ldo = N; s.po = (long long)M * N; s.out_rows = M; s.out_cols = N;
      s.e2h = h2 ? &rec[2].e : nullptr;
      split_planes(s, false, 1, nullptr);
    }
  }
  SplitGemmParams g{};
  g.A = Ap; g.lda = Kp; g.pA = (long long)M * Kp; g.sA = 3 * g.pA;
  g.B = Bp; g.ldb = Kp; g.pB = (long long)N * Kp; g.sB = 3 * g.pB;
  g.b_frag = bfrag ? 1 : 0;
  g.C = dC; g.ldc = N; g.sC = (long long)M * N;
  g.bias = dbias; g.sBias = N;
  g.mask = dmask; g.ldm = N; g.sMask = (long long)M * N;
  if (m16) {
    g.mask16 = dM16;
    g.sMask = 3ll * M * N;
  }
  if (Csum) {
    g.Cp = dCp; g.ldcp = N; g.pC = (long long)M * N; g.sCp = 3 * g.pC;
  }
  g.M = M; g.N = N; g.K = (int)Kp;
  g.np = h2 ? 2 : np;
  if (h2) {
    g.ra = rec + 0; g.na = 1;
    g.rb = rec + 1; g.nb = 1;
    g.rc = rec + 3;
    g.bias_in_b = epi == 1 && bias ? 1 : 0;
    g.pMask = (long long)M * N;
    g.kmul = (float)K;
  }
  if (autosplit) {
    g.ws = d.get<float>((size_t)std::max(gemm_x3f_ws_floats(M, N, (int)Kp, batch), 1LL));
    if (!g.ws) return -12;
    g.splits = -1;
    if (fin) {
      g.cnt = d.get<int>((size_t)GEMM_X3F_CNT);
      if (!g.cnt || hipMemset(g.cnt, 0, sizeof(int) * GEMM_X3F_CNT) != hipSuccess) return -12;
    }
  }
  if (small) {
    if (!gemm_x3s_ok(g, epi, batch)) return -95;
    gemm_x3s(g, epi, batch, nullptr);
  } else {
    if (!gemm_x3f_ok(g, epi, batch)) return -95;
    gemm_x3f(g, epi, batch, nullptr);
  }
  {
    const hipError_t le = hipGetLastError();  // a launch the runtime refused leaves C as it was
    if (le != hipSuccess) {
      fprintf(stderr, "[mtsac_debug_gemm_x3f] launch refused: %s\n", hipGetErrorString(le));
      return -6;
    }
  }
  if (hipDeviceSynchronize() != hipSuccess) return -5;
  if (hipMemcpy(C, dC, sizeof(float) * nC, hipMemcpyDeviceToHost) != hipSuccess) return -5;
  if (Csum && h2) {  // (h + l) 2^-ec
    std::vector<_Float16> h(3 * nC);
    int ec = 0;
    if (hipMemcpy(h.data(), dCp, sizeof(_Float16) * h.size(), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&ec, &rec[3].e, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
      return -5;
    const size_t n = (size_t)M * N;
    for (int z = 0; z < batch; ++z)
      for (size_t i = 0; i < n; ++i) {
        const _Float16* q = &h[(size_t)z * 3 * n];
        Csum[(size_t)z * n + i] = std::ldexp((float)q[i] + (float)q[n + i], -ec);
      }
  } else if (Csum) {
    std::vector<__bf16> h(3 * nC);
    if (hipMemcpy(h.data(), dCp, sizeof(__bf16) * h.size(), hipMemcpyDeviceToHost) != hipSuccess) return -5;
    const size_t n = (size_t)M * N;
    for (int z = 0; z < batch; ++z)
      for (size_t i = 0; i < n; ++i) {
        const __bf16* q = &h[(size_t)z * 3 * n];
        Csum[(size_t)z * n + i] = ((float)q[i] + (float)q[n + i]) + (float)q[2 * n + i];
      }
  }
  return 0;
}

// time iters launches of the forward-shaped plane GEMM (C = relu(A . B^T + bias) with planes out)
// on device-resident random planes; which: 0 = gemm_x3p (row-major A, k-major B: the engine's
// current forward), 1 = gemm_x3f (row-major both)
int mtsac_debug_gemm_fwd_bench(int which, int epi, int batch, int M, int N, int K, int iters, double* ms_per_launch) {
  const int outs = (epi >> 8) & 3;  // 0: fp32 + planes, 1: planes only, 2: fp32 only
  const int np = ((epi >> 10) & 1) ? 1 : 3;  // bf16: the high plane only
  const bool autosplit = (epi >> 11) & 1;     // split-K by the launcher's own choice (workspace given)
  const bool fin = (epi >> 12) & 1;           // ... with arrival counters: the in-launch finish
  const bool h2 = (epi >> 13) & 1;            // precision split2h (exponents 0: operands in [-1, 1])
  const bool bfrag = (epi >> 14) & 1;         // gemm_x3f: B planes in the fragment layout
  epi &= 255;
  if (M < 1 || N < 1 || K < 1 || batch < 1 || iters < 1 || !ms_per_launch) return -22;
  DevBuf d;
  const long long Kp = (K + 63) / 64 * 64;
  PlaneRec* rec = d.get<PlaneRec>(3);  // zero exponents: the random operands lie in [-1, 1]
  if (!rec) return -12;
  float* fa = d.get<float>((size_t)M * Kp);
  float* fb = d.get<float>((size_t)N * Kp);
  float* C = d.get<float>((size_t)M * N * batch);
  float* bias = d.get<float>((size_t)N * batch);
  __bf16* Cp = d.get<__bf16>((size_t)3 * M * N * batch);
  if (!fa || !fb || !C || !bias || !Cp) return -12;
  hipLaunchKernelGGL(fill_rand_f32, dim3((unsigned)(((long long)M * Kp + 255) / 256)), dim3(256), 0, nullptr, fa,
                     (long long)M * Kp, 3u);
  hipLaunchKernelGGL(fill_rand_f32, dim3((unsigned)(((long long)N * Kp + 255) / 256)), dim3(256), 0, nullptr, fb,
                     (long long)N * Kp, 5u);
  const bool bk = which == 0;  // gemm_x3p forward: B k-major [K][N]
  long long lda, pa, ldb, pb;
  plane_geom(M, (int)Kp, false, lda, pa);
  plane_geom(N, (int)Kp, bk, ldb, pb);
  __bf16* Ap = d.get<__bf16>((size_t)3 * pa * batch);
  __bf16* Bp = d.get<__bf16>((size_t)3 * pb * batch);
  if (!Ap || !Bp) return -12;
  for (int z = 0; z < batch; ++z) {
    split_into(fa, M, (int)Kp, false, Ap + 3 * pa * z, h2 ? &rec[0].e : nullptr);
    split_into(fb, N, (int)Kp, bk, Bp + 3 * pb * z, h2 ? &rec[1].e : nullptr, bfrag && !bk);
  }
  SplitGemmParams g{};
  if (h2) {
    g.ra = rec; g.rb = rec + 1; g.rc = rec + 2;
    g.kmul = (float)K;
    g.pMask = (long long)M * N;
  }
  g.A = Ap; g.lda = lda; g.pA = pa; g.sA = 3 * pa;
  g.B = Bp; g.ldb = ldb; g.pB = pb; g.sB = 3 * pb; g.b_kmajor = bk;
  g.b_frag = bfrag && !bk ? 1 : 0;
  g.C = C; g.ldc = N; g.sC = (long long)M * N;
  g.bias = bias; g.sBias = N;
  g.mask = C; g.ldm = N; g.sMask = (long long)M * N;
  g.Cp = Cp; g.ldcp = N; g.pC = (long long)M * N; g.sCp = 3 * g.pC;
  if (outs == 1) g.C = nullptr;
  if (outs == 2) g.Cp = nullptr;
  g.M = M; g.N = N; g.K = (int)Kp;
  g.splits = 1;
  g.np = h2 ? 2 : np;
  if (autosplit) {
    const long long wsf = std::max(gemm_x3f_ws_floats(M, N, (int)Kp, batch), gemm_x3p_ws_floats(M, N, (int)Kp, batch, false));
    g.ws = d.get<float>((size_t)std::max(wsf, 1LL));
    if (!g.ws) return -12;
    g.splits = -1;
    if (fin) {
      g.cnt = d.get<int>((size_t)GEMM_X3F_CNT);
      if (!g.cnt) return -12;
    }
  }
  if (which >= 1 && !gemm_x3f_ok(g, epi, batch)) return -95;
  if (which < 0 && !gemm_x3s_ok(g, epi, batch)) return -95;
  auto run = [&]() {
    if (which == -1) gemm_x3s(g, epi, batch, nullptr);
    else if (which < -1) gemm_x3s_ablate(g, -1 - which, batch, nullptr);  // -2 no loads, -3 no MFMAs
    else if (which >= 2) gemm_x3f_ablate(g, which - 2, batch, nullptr);  // 2 + ablation bits (planes out)
    else if (which == 1) gemm_x3f(g, epi, batch, nullptr);
    else gemm_x3p(g, epi, batch, nullptr);
  };
  run();
  hipEvent_t e0, e1;
  if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return -5;
  (void)hipEventRecord(e0, nullptr);
  for (int i = 0; i < iters; ++i) run();
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
  if (geo < 0) {  // restore the default (e.g. the value this function returned)
    g_x3p_geo = -1;
    g_x3p_dbg = g_x3_dbg = 0;
    return old;
  }
  const int g = geo & 255;
  g_x3p_geo = g <= 5 ? g : -1;
  g_x3p_dbg = (geo >> 8) & 255;
  g_x3_dbg = (geo >> 16) & 255;
  return old;
}

int mtsac_debug_x3s_ti(int M, int N, int batch) { return gemm_x3s_ti(M, N, batch); }

// DrQ conv channel groups per lane (0 = the engine's choice); returns the previous fwd | bwd << 8
int mtsac_debug_drq_groups(int fwd, int bwd) {
  const int old = drq::g_drq_fwd_g | (drq::g_drq_bwd_g << 8);
  drq::g_drq_fwd_g = fwd;
  drq::g_drq_bwd_g = bwd;
  return old;
}

// DrQ convs on f32 MFMA (bit 1 forward, 2 data grad, 4 weight grad) or the VALU kernels; returns the
// previous mask (< 0: query only)
int mtsac_debug_drq_mfma(int mask) {
  const int old = drq::g_drq_mfma;
  if (mask >= 0) drq::g_drq_mfma = mask & 7;
  return old;
}

// the pre-round-6 DrQ conv kernels (bit 1 forward, 2 data grad, 4 weight grad) or the row-tile ones;
// returns the previous mask (< 0: query only)
int mtsac_debug_drq_legacy(int mask) {
  const int old = drq::g_drq_legacy;
  if (mask >= 0) drq::g_drq_legacy = mask & 63;
  return old;
}

// the row-tile conv weight grad's grid cap (> 0 sets, 0 restores the per-shape default; < 0 queries;
// returns the previous); engines created before a change keep partial buffers sized for the old cap,
// so set it before creating one (experiments)
int mtsac_debug_drq_wgrad_blocks(int cap) {
  const int old = drq::g_drq_wg_blocks;
  if (cap >= 0) drq::g_drq_wg_blocks = cap;
  return old;
}

// mean microseconds per launch of one DrQ conv pass on random operands (drq::conv_bench)
int mtsac_debug_drq_conv_bench(int kind, int B, int H, int W, int ci, int co, int iters, double* us_per_launch) {
  if (kind < 0 || kind > 2 || B < 1 || H < 1 || W < 1 || iters < 1 || !us_per_launch || !drq::conv_supported(ci, co))
    return -22;
  const double us = drq::conv_bench(kind, B, H, W, ci, co, iters);
  if (us < 0) return -12;
  *us_per_launch = us;
  return hipDeviceSynchronize() == hipSuccess ? 0 : -5;
}

}  // extern "C"
