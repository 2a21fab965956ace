// layout.hip -- split-K reduction and fp32 transposes for the GEMM launchers (gfx950).
#include <algorithm>

#include "kernels.h"

namespace mtsac {

namespace {

constexpr int BK = 32;          // K-tile of both GEMM kernels: slices are whole K-tiles
constexpr int TARGET_WG = 512;  // two 256-thread workgroups per CU on 256 CUs

// C[z][m][n] = sum_s ws[z*S+s][m][n] in slice order (float4 over n when aligned)
__global__ void splitk_reduce_kernel(const float* __restrict__ ws, int S, int M, int N, float* __restrict__ C, int ldc,
                                     long long sC) {
  const int z = blockIdx.y;
  const long long slab = (long long)M * N;
  const float* w = ws + (long long)z * S * slab;
  float* c = C + z * sC;
  const long long n4 = slab / 4;
  const bool vec = (N % 4 == 0) && (ldc % 4 == 0);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < (vec ? n4 : slab);
       i += (long long)gridDim.x * blockDim.x) {
    if (vec) {
      float4 acc = reinterpret_cast<const float4*>(w)[i];
      for (int s = 1; s < S; ++s) {
        const float4 v = reinterpret_cast<const float4*>(w + s * slab)[i];
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
      const long long e = 4 * i, m = e / N, n = e - m * N;
      *reinterpret_cast<float4*>(c + m * ldc + n) = acc;
    } else {
      float acc = w[i];
      for (int s = 1; s < S; ++s) acc += w[s * slab + i];
      const long long m = i / N, n = i - m * N;
      c[m * ldc + n] = acc;
    }
  }
}

// One launch for everything that follows a split-K weight gradient: blocks [0, nred) reduce the
// slabs into C (as splitk_reduce_kernel), [nred, nred + ndb) add the per-slice bias sums (as
// splitk_db_kernel), the rest finish the bias grad from column-sum partials (as colsum_final_kernel,
// 64 columns per block): the same sums in the same order, two or three launches fewer per layer.
__device__ inline void finish_job(const ReduceJob& j, int nred, int ndb, int bx, int z) {
  if (bx < nred) {
    const long long slab = (long long)j.M * j.N;
    const float* w = j.ws + (long long)z * j.S * slab;
    float* c = j.C + z * j.sC;
    const long long n4 = slab / 4;
    const bool vec = (j.N % 4 == 0) && (j.ldc % 4 == 0);
    for (long long i = (long long)bx * 256 + threadIdx.x; i < (vec ? n4 : slab); i += (long long)nred * 256) {
      if (vec) {
        float4 acc = reinterpret_cast<const float4*>(w)[i];
        for (int s = 1; s < j.S; ++s) {
          const float4 v = reinterpret_cast<const float4*>(w + s * slab)[i];
          acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        }
        const long long e = 4 * i, m = e / j.N, n = e - m * j.N;
        *reinterpret_cast<float4*>(c + m * j.ldc + n) = acc;
      } else {
        float acc = w[i];
        for (int s = 1; s < j.S; ++s) acc += w[s * slab + i];
        const long long m = i / j.N, n = i - m * j.N;
        c[m * j.ldc + n] = acc;
      }
    }
    return;
  }
  if (bx < nred + ndb) {
    const int n = (bx - nred) * 256 + threadIdx.x;
    if (n >= j.N) return;
    const float* w = j.dbws + (long long)z * j.S * j.N;
    float acc = w[n];
    for (int s = 1; s < j.S; ++s) acc += w[(long long)s * j.N + n];
    j.db[z * j.sDb + n] = acc;
    return;
  }
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = (bx - nred - ndb) * 64 + cl;
  const int cols = j.N, chunks = j.cs_chunks;
  float s = 0.f;
  if (c < cols) {
    const float* pz = j.cs_part + (long long)z * chunks * cols + c;
    int ch = g;
    for (; ch + 28 < chunks; ch += 32) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = pz[(long long)(ch + 4 * u) * cols];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; ch < chunks; ch += 4) s += pz[(long long)ch * cols];
  }
  red[g][cl] = s;
  __syncthreads();
  if (g == 0 && c < cols) j.cs_db[z * j.cs_sdb + c] = ((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl];
}

__global__ __launch_bounds__(256) void splitk_finish_all_kernel(ReduceJob j, int nred, int ndb) {
  finish_job(j, nred, ndb, blockIdx.x, blockIdx.y);
}

// the jobs of a FinishSink: job k owns blocks [start[k], start[k + 1]) (block-uniform branch)
struct FinishJobs {
  DeferredFinish job[FINISH_SINK_JOBS];
  int start[FINISH_SINK_JOBS + 1];
  int n;
};
__global__ __launch_bounds__(256) void splitk_finish_many_kernel(FinishJobs js) {
  const int bx = blockIdx.x;
  int k = 0;
  while (k + 1 < js.n && bx >= js.start[k + 1]) ++k;
  finish_job(js.job[k].j, js.job[k].nred, js.job[k].ndb, bx - js.start[k], blockIdx.y);
}

__global__ void splitk_db_kernel(const float* __restrict__ dbws, int S, int N, float* __restrict__ db, long long sDb) {
  const int z = blockIdx.y;
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const float* w = dbws + (long long)z * S * N;
  float acc = w[n];
  for (int s = 1; s < S; ++s) acc += w[(long long)s * N + n];
  db[z * sDb + n] = acc;
}

// 64 x 64 tiles through LDS (+1 column of padding: conflict-free both ways)
__global__ __launch_bounds__(256) void transpose_kernel(const float* __restrict__ in, long long s_in,
                                                        float* __restrict__ out, long long s_out, int rows, int cols) {
  __shared__ float t[64][65];
  const int z = blockIdx.z;
  const float* src = in + z * s_in;
  float* dst = out + z * s_out;
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int r = r0 + i, c = c0 + tx;
    t[i][tx] = (r < rows && c < cols) ? src[(long long)r * cols + c] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int c = c0 + i, r = r0 + tx;
    if (c < cols && r < rows) dst[(long long)c * rows + r] = t[tx][i];
  }
}

}  // namespace

int gemm_splits(int M, int N, int K, int batch) {
  const long long tiles = (long long)((M + 127) / 128) * ((N + 127) / 128) * batch;
  if (tiles >= TARGET_WG) return 1;
  const int kt = (K + BK - 1) / BK;
  int s = (int)((TARGET_WG + tiles - 1) / tiles);
  s = std::min(s, 16);
  s = std::min(s, std::max(1, kt / 4));  // keep >= 4 K-tiles per slice
  return std::max(s, 1);
}

long long gemm_ws_floats(int M, int N, int batch, int splits) {
  if (splits <= 1) return 0;
  return (long long)batch * splits * ((long long)M * N + N);
}

DeferredFinish reduce_job(const GemmParams& p, int batch, int splits, const float* cs_part, int cs_chunks,
                          float* cs_db, long long cs_sdb) {
  const long long slab = (long long)p.M * p.N;
  const long long work = (p.N % 4 == 0 && p.ldc % 4 == 0) ? slab / 4 : slab;
  DeferredFinish d{};
  d.nred = std::max(1, (int)std::min<long long>((work + 255) / 256, 1024));
  ReduceJob& j = d.j;
  j.ws = p.ws; j.S = splits; j.M = p.M; j.N = p.N; j.C = p.C; j.ldc = p.ldc; j.sC = p.sC;
  if (p.db) {
    j.dbws = p.ws + (long long)batch * splits * slab;
    j.db = p.db;
    j.sDb = p.sDb;
    d.ndb = (p.N + 255) / 256;
  }
  if (cs_part && cs_chunks > 0) {
    j.cs_part = cs_part; j.cs_chunks = cs_chunks; j.cs_db = cs_db; j.cs_sdb = cs_sdb;
    d.ncs = (p.N + 63) / 64;
  }
  return d;
}

DeferredFinish colsum_job(const float* part, int cols, int chunks, float* db, long long sdb) {
  DeferredFinish d{};
  d.j.N = cols;
  d.j.cs_part = part; d.j.cs_chunks = chunks; d.j.cs_db = db; d.j.cs_sdb = sdb;
  d.ncs = (cols + 63) / 64;
  return d;
}

void finish_many(FinishSink& s, int batch, hipStream_t st) {
  if (s.n <= 0) return;
  FinishJobs js{};
  js.n = s.n;
  int b = 0;
  for (int k = 0; k < s.n; ++k) {
    js.job[k] = s.job[k];
    js.start[k] = b;
    b += s.job[k].nred + s.job[k].ndb + s.job[k].ncs;
  }
  js.start[s.n] = b;
  s.n = 0;
  if (b > 0) hipLaunchKernelGGL(splitk_finish_many_kernel, dim3(b, batch), dim3(256), 0, st, js);
}

void splitk_reduce(const GemmParams& p, int batch, int splits, hipStream_t st, const float* cs_part, int cs_chunks,
                   float* cs_db, long long cs_sdb) {
  const DeferredFinish d = reduce_job(p, batch, splits, cs_part, cs_chunks, cs_db, cs_sdb);
  hipLaunchKernelGGL(splitk_finish_all_kernel, dim3(d.nred + d.ndb + d.ncs, batch), dim3(256), 0, st, d.j, d.nred,
                     d.ndb);
}

void transpose_f32(const float* in, long long s_in, float* out, long long s_out, int rows, int cols, int batch,
                   hipStream_t st) {
  if (rows <= 0 || cols <= 0 || batch <= 0) return;
  hipLaunchKernelGGL(transpose_kernel, dim3((cols + 63) / 64, (rows + 63) / 64, batch), dim3(256), 0, st, in, s_in, out,
                     s_out, rows, cols);
}

}  // namespace mtsac
