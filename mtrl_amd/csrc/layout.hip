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

void splitk_reduce(const GemmParams& p, int batch, int splits, hipStream_t st) {
  const long long slab = (long long)p.M * p.N;
  const long long work = (p.N % 4 == 0 && p.ldc % 4 == 0) ? slab / 4 : slab;
  const int blocks = (int)std::min<long long>((work + 255) / 256, 1024);
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(std::max(blocks, 1), batch), dim3(256), 0, st, p.ws, splits, p.M,
                     p.N, p.C, p.ldc, p.sC);
  if (p.db)
    hipLaunchKernelGGL(splitk_db_kernel, dim3((p.N + 255) / 256, batch), dim3(256), 0, st,
                       p.ws + (long long)batch * splits * slab, splits, p.N, p.db, p.sDb);
}

void transpose_f32(const float* in, long long s_in, float* out, long long s_out, int rows, int cols, int batch,
                   hipStream_t st) {
  if (rows <= 0 || cols <= 0 || batch <= 0) return;
  hipLaunchKernelGGL(transpose_kernel, dim3((cols + 63) / 64, (rows + 63) / 64, batch), dim3(256), 0, st, in, s_in, out,
                     s_out, rows, cols);
}

}  // namespace mtsac
