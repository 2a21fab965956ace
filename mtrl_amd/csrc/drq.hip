// drq.hip -- the DrQ-eps update path (distributional dueling DQN on an IMPALA CNN) for gfx950.
//
// Reference: mtrl/rl/algorithms/drqeps.py:268-335 (_update_inner), mtrl/nn/impala.py:13-48,
// mtrl/rl/networks.py:99-149, mtrl/nn/augmentation.py:36-117, mtrl/nn/task_embedding.py:5-12.
//
// Shapes are tiny (3x3 convs with 4-16 channels on 84x84 -> 11x11 NHWC images, 26 games, batch
// 256): every conv here is a direct convolution, one lane per output (or input) pixel with all of
// that pixel's channels in registers and the 3x3 x Cin x Cout weights in LDS (read as broadcasts).
// These passes are bound by the per-CU LDS/VALU issue of the weight broadcasts and the L2-served
// neighbour reads, not by HBM or MFMA (Cout <= 16 leaves MFMA tiles mostly empty); the dense head
// runs on gemm_f32 (exact fp32).  Weight gradients reduce over batch x pixels into per-block
// partials summed in a fixed order (bitwise reproducible).
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "drq_kernels.h"

namespace mtsac {
namespace drq {

namespace {

__device__ inline float wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ inline float wmax(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// ------------------------------------------------------------------ augmentation
// augment (augmentation.py:101-117) with its draws given: uint8 [B][C][H][W] -> NHWC float in
// [-1, 1], edge pad 4 (= clamped reads), crop at (ox, oy), times the intensity factor.
__global__ void augment_kernel(const unsigned char* __restrict__ obs, const int* __restrict__ crop,
                               const float* __restrict__ noise, float* __restrict__ out, int B, int C, int H, int W,
                               int pad) {
  // 32-bit indexing: B H W C < 2^31 (checked at drq_create)
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * H * W * C) return;
  int r = i / C;
  const int c = i - r * C;
  int r2 = r / W;
  const int x = r - r2 * W;
  r = r2 / H;
  const int y = r2 - r * H;
  const int b = r;
  const int sy = min(max(y + crop[2 * b] - pad, 0), H - 1);
  const int sx = min(max(x + crop[2 * b + 1] - pad, 0), W - 1);
  const float v = (float)obs[(((long long)b * C + c) * H + sy) * W + sx];
  out[i] = ((v / 255.0f - 0.5f) * 2.0f) * noise[b];
}

// the update's 3B-image input [s | s' | s'] in one launch: element i < n of the obs half and its
// next-obs twin, the augmented next obs written twice (online and target rows of the encoder pass)
__global__ void augment3_kernel(const unsigned char* __restrict__ obs, const int* __restrict__ crop_o,
                                const float* __restrict__ noise_o, const unsigned char* __restrict__ nobs,
                                const int* __restrict__ crop_n, const float* __restrict__ noise_n,
                                float* __restrict__ out, int B, int C, int H, int W, int pad) {
  // one lane per output pixel (all C channels: one index decomposition, C byte loads in flight, a
  // float4 store per 4 channels); the arithmetic per element is augment_kernel's
  const int np = B * H * W;  // B H W C < 2^31 (checked at drq_create)
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * np) return;
  const bool next = i >= np;
  if (next) i -= np;
  const unsigned char* src = next ? nobs : obs;
  const int* crop = next ? crop_n : crop_o;
  const float* noise = next ? noise_n : noise_o;
  int r = i / W;
  const int x = i - r * W;
  const int b = r / H;
  const int y = r - b * H;
  const int sy = min(max(y + crop[2 * b] - pad, 0), H - 1);
  const int sx = min(max(x + crop[2 * b + 1] - pad, 0), W - 1);
  const unsigned char* sp = src + ((long long)b * C * H + sy) * W + sx;  // channel c at sp + c H W
  const float f = noise[b];
  const long long o = (long long)i * C, n = (long long)np * C;
  auto put = [&](long long k, float v) {
    if (next) {
      out[n + k] = v;
      out[2 * n + k] = v;
    } else {
      out[k] = v;
    }
  };
  if (C == 4) {
    float4 v;
    v.x = (((float)sp[0] / 255.0f - 0.5f) * 2.0f) * f;
    v.y = (((float)sp[(long long)H * W] / 255.0f - 0.5f) * 2.0f) * f;
    v.z = (((float)sp[2LL * H * W] / 255.0f - 0.5f) * 2.0f) * f;
    v.w = (((float)sp[3LL * H * W] / 255.0f - 0.5f) * 2.0f) * f;
    if (next) {
      *reinterpret_cast<float4*>(out + n + o) = v;
      *reinterpret_cast<float4*>(out + 2 * n + o) = v;
    } else {
      *reinterpret_cast<float4*>(out + o) = v;
    }
  } else {
    for (int c = 0; c < C; ++c) put(o + c, (((float)sp[(long long)c * H * W] / 255.0f - 0.5f) * 2.0f) * f);
  }
}

// ------------------------------------------------------------------ Atari replay sample
// MemoryEfficientAtariMultiTaskReplayBuffer.sample (buffers.py:1188-1227) from the device store:
// row b = (sample i = b / T, task t = b % T); draw k = idx[i] -> slot via the guard window
// (_sample_indices, buffers.py:1082-1105); next_obs = the frame stack nstep slots ahead; rewards
// min-max normalised in double per task; task_ids as the reference lists them (b / n).
// Row mode (rslot != null, sample_unbalanced, buffers.py:1230-1279): row b reads slot rslot[b] of
// task rtask[b], both drawn on the host, and task_ids = rtask[b].
// AtariMultiTaskReplayBuffer (nstore != null): next_obs from its own array at the same slot.
struct AtariSampleParams {
  const unsigned char* store;  // [cap][T][img]
  const unsigned char* nstore; // [cap][T][img] next_obs (buffer kind 1) or null
  const int* act;
  const float *rew, *done, *trunc;  // [cap][T]
  const double* minmax;        // [2][T] (normalize) or null
  const int* idx;
  long long cap;
  int T, n, img16, nstep, full, pos, guard;
  double eps;
  unsigned char *obs, *nobs;
  int *act_out, *task_out;
  float *rew_out, *done_out, *trunc_out;
  const long long* rslot;
  const int* rtask;
};

__global__ void atari_sample_kernel(AtariSampleParams p) {
  const int b = blockIdx.y;
  int i = b / p.T, t = b - i * p.T;
  long long slot = p.rslot ? p.rslot[b] : p.idx[i];
  if (p.rslot) t = p.rtask[b];
  else if (p.full) {
    const long long k = slot;
    if (p.pos + p.guard <= p.cap) slot = k < p.pos ? k : k + p.guard;
    else slot = k + (p.pos + p.guard - p.cap);
  }
  const long long nslot = p.nstore ? slot : (slot + p.nstep) % p.cap;
  const uint4* src = reinterpret_cast<const uint4*>(p.store) + (slot * p.T + t) * p.img16;
  const uint4* nsrc = reinterpret_cast<const uint4*>(p.nstore ? p.nstore : p.store) + (nslot * p.T + t) * p.img16;
  uint4* dst = reinterpret_cast<uint4*>(p.obs) + (long long)b * p.img16;
  uint4* ndst = reinterpret_cast<uint4*>(p.nobs) + (long long)b * p.img16;
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < p.img16; c += gridDim.x * blockDim.x) {
    dst[c] = src[c];
    ndst[c] = nsrc[c];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const long long r = slot * p.T + t;
    p.act_out[b] = p.act[r];
    float rw = p.rew[r];
    if (p.minmax) {
      const double mn = p.minmax[t], mx = p.minmax[p.T + t];
      if (p.nstore) {  // (rewards - mn) / (mx - mn + eps) in float64, one rounding (buffers.py:877)
        rw = (float)(((double)rw - mn) / (mx - mn + p.eps));
      } else {  // rewards -= mn; rewards /= (...): in place on float32 (buffers.py:1207-1212)
        rw = (float)((double)rw - mn);
        rw = (float)((double)rw / (mx - mn + p.eps));
      }
    }
    p.rew_out[b] = rw;
    p.done_out[b] = p.done[r];
    p.trunc_out[b] = p.trunc[r];
    p.task_out[b] = p.rslot ? t : b / p.n;  // np.repeat(np.arange(T), n)
  }
}

// ------------------------------------------------------------------ augmentation draws
// The device-side draws of the sample+update entries (the reference takes them from jax.random,
// augmentation.py:75-117; threefry is not reproduced): per row two crop offsets in [0, 2 pad) and
// an intensity factor 1 + 0.05 clip(N(0, 1), -2, 2), for obs and next_obs, from a counter hash.
__device__ inline unsigned long long mix64(unsigned long long z) {
  z += 0x9e3779b97f4a7c15ULL;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

__global__ void aug_draw_kernel(unsigned long long seed, unsigned long long ctr, int B, int span, int* crop_o,
                                float* noise_o, int* crop_n, float* noise_n) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= 2 * B) return;
  const unsigned long long h0 = mix64(seed ^ mix64(ctr * 0x100000001b3ULL + (unsigned long long)b));
  const unsigned long long h1 = mix64(h0 ^ 0x5851f42d4c957f2dULL);
  const int r = b < B ? b : b - B;
  int* crop = b < B ? crop_o : crop_n;
  float* noise = b < B ? noise_o : noise_n;
  crop[2 * r] = (int)((h0 & 0xffffffffULL) % (unsigned)span);
  crop[2 * r + 1] = (int)((h0 >> 32) % (unsigned)span);
  const float u1 = ((float)(h1 >> 40) + 0.5f) * (1.0f / 16777216.0f);  // (0, 1)
  const float u2 = (float)((h1 >> 16) & 0xffffffULL) * (1.0f / 16777216.0f);
  const float z = sqrtf(-2.0f * logf(u1)) * cosf(6.283185307179586f * u2);
  noise[r] = 1.0f + 0.05f * fminf(fmaxf(z, -2.0f), 2.0f);
}

// ------------------------------------------------------------------ convolutions
// out[b][y][x][:] = bias + sum_{dy,dx,ci} act(in[b][y+dy-1][x+dx-1][ci]) w[dy][dx][ci][:]
// (+ res[b][y][x][:]); act = relu when RELU_IN.  One lane per (output pixel, group of CG output
// channels), the group uniform over the block (blockIdx.y).  The weights are read straight from
// global memory with wave-uniform addresses, so they arrive by scalar loads as SGPR operands of
// packed FMAs (an LDS copy put a broadcast read in front of every four FMAs).  The per-output
// summation order (taps, then input channels) does not depend on CG.
template <int CI, int CO, int CG, bool RELU_IN, bool ADD_RES>
__global__ __launch_bounds__(256) void conv_fwd_kernel(const float* __restrict__ in, const float* __restrict__ w_a,
                                                       const float* __restrict__ bias_a,
                                                       const float* __restrict__ w_b,
                                                       const float* __restrict__ bias_b, const float* __restrict__ res,
                                                       float* __restrict__ out, int B, int B1, int H, int W) {
  // images [0, B1) use (w_a, bias_a), [B1, B) (w_b, bias_b): the blocks of the two ranges are
  // separate, so the weights stay block-uniform (scalar loads)
  const int cg = blockIdx.y * CG;
  const int n1 = B1 * H * W, nb1 = (n1 + 255) / 256;
  const bool second = (int)blockIdx.x >= nb1;
  const int pix = second ? n1 + ((int)blockIdx.x - nb1) * 256 + (int)threadIdx.x : (int)blockIdx.x * 256 + (int)threadIdx.x;
  if (pix >= (second ? B * H * W : n1)) return;
  const float* __restrict__ w = second ? w_b : w_a;
  const float* __restrict__ bias = second ? bias_b : bias_a;
  const int x = pix % W, y = (pix / W) % H;
  float acc[CG];
#pragma unroll
  for (int c = 0; c < CG; ++c) acc[c] = bias[cg + c];
#pragma unroll
  for (int dy = 0; dy < 3; ++dy) {
    const int yy = y + dy - 1;
    if (yy < 0 || yy >= H) continue;
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      const int xx = x + dx - 1;
      if (xx < 0 || xx >= W) continue;
      const float* ip = in + (long long)(pix + (dy - 1) * W + (dx - 1)) * CI;
      float v[CI];
#pragma unroll
      for (int c4 = 0; c4 < CI; c4 += 4) {
        const float4 q = *reinterpret_cast<const float4*>(ip + c4);
        v[c4] = q.x; v[c4 + 1] = q.y; v[c4 + 2] = q.z; v[c4 + 3] = q.w;
      }
      const float* wt = w + (dy * 3 + dx) * CI * CO + cg;
#pragma unroll
      for (int ci = 0; ci < CI; ++ci) {
        const float a = RELU_IN ? fmaxf(v[ci], 0.f) : v[ci];
#pragma unroll
        for (int c = 0; c < CG; ++c) acc[c] = fmaf(a, wt[ci * CO + c], acc[c]);
      }
    }
  }
  float* op = out + (long long)pix * CO + cg;
#pragma unroll
  for (int c4 = 0; c4 < CG; c4 += 4) {
    float4 o = make_float4(acc[c4], acc[c4 + 1], acc[c4 + 2], acc[c4 + 3]);
    if (ADD_RES) {
      const float4 r = *reinterpret_cast<const float4*>(res + (long long)pix * CO + cg + c4);
      o.x += r.x; o.y += r.y; o.z += r.z; o.w += r.w;
    }
    *reinterpret_cast<float4*>(op + c4) = o;
  }
}

// din[b][y][x][ci] = (sum_{dy,dx,co} dout[b][y-dy+1][x-dx+1][co] w[dy][dx][ci][co]) * [mask > 0]
// (MASK: the ReLU in front of the conv) (+ dres[b][y][x][ci]).  One lane per (input pixel, group
// of CG input channels), weights by scalar loads as above.
template <int CI, int CO, int CG, bool MASK, bool ADD_RES>
__global__ __launch_bounds__(256) void conv_bwd_data_kernel(const float* __restrict__ dout, const float* __restrict__ w,
                                                            const float* __restrict__ mask,
                                                            const float* __restrict__ dres, float* __restrict__ din,
                                                            int B, int H, int W) {
  const int cg = blockIdx.y * CG;
  const int pix = blockIdx.x * 256 + threadIdx.x;
  if (pix >= B * H * W) return;
  const int x = pix % W, y = (pix / W) % H;
  float acc[CG];
#pragma unroll
  for (int c = 0; c < CG; ++c) acc[c] = 0.f;
#pragma unroll
  for (int dy = 0; dy < 3; ++dy) {
    const int yy = y - dy + 1;
    if (yy < 0 || yy >= H) continue;
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      const int xx = x - dx + 1;
      if (xx < 0 || xx >= W) continue;
      const float* gp = dout + (long long)(pix + (1 - dy) * W + (1 - dx)) * CO;
      float g[CO];
#pragma unroll
      for (int c4 = 0; c4 < CO; c4 += 4) {
        const float4 q = *reinterpret_cast<const float4*>(gp + c4);
        g[c4] = q.x; g[c4 + 1] = q.y; g[c4 + 2] = q.z; g[c4 + 3] = q.w;
      }
      const float* wt = w + (dy * 3 + dx) * CI * CO + cg * CO;
#pragma unroll
      for (int c = 0; c < CG; ++c) {
        float s = acc[c];
#pragma unroll
        for (int co = 0; co < CO; ++co) s = fmaf(g[co], wt[c * CO + co], s);
        acc[c] = s;
      }
    }
  }
#pragma unroll
  for (int c4 = 0; c4 < CG; c4 += 4) {
    const long long o = (long long)pix * CI + cg + c4;
    float4 r4 = make_float4(acc[c4], acc[c4 + 1], acc[c4 + 2], acc[c4 + 3]);
    if (MASK) {
      const float4 m = *reinterpret_cast<const float4*>(mask + o);
      r4.x = m.x > 0.f ? r4.x : 0.f; r4.y = m.y > 0.f ? r4.y : 0.f;
      r4.z = m.z > 0.f ? r4.z : 0.f; r4.w = m.w > 0.f ? r4.w : 0.f;
    }
    if (ADD_RES) {
      const float4 r = *reinterpret_cast<const float4*>(dres + o);
      r4.x += r.x; r4.y += r.y; r4.z += r.z; r4.w += r.w;
    }
    *reinterpret_cast<float4*>(din + o) = r4;
  }
}

// Weight gradient partials: block g takes 64-pixel tiles g, g + G, ... (G = gridDim.x); the
// tile's im2col rows (act applied, zero outside the image) and dout go through LDS; lane t owns a
// 4 x 4 block of dW ([tap * CI + ci][co]) over the pixels q = pg, pg + PG, ... of every tile (PG
// lane groups when the blocks leave lanes over), the groups' partials summed in group order at
// the end; the bias entries are summed by 256 / CO lane groups over interleaved pixels, the groups
// added in order at the end.  part[g][9 CI CO + CO], summed over g in order by sum_parts_kernel.
template <int CI, int CO, bool RELU_IN>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(const float* __restrict__ in, const float* __restrict__ dout,
                                                         float* __restrict__ part, int B, int H, int W) {
  constexpr int NW = 9 * CI * CO;
  constexpr int NB = (9 * CI / 4) * (CO / 4);  // 4 x 4 blocks of dW ([tap * CI + ci][co])
  constexpr int PG = 256 / NB;                 // pixel groups: lane t = (pg, blk), q = pg, pg + PG, ...
  constexpr int TP = 64;
  __shared__ float sin_[TP][9 * CI];
  __shared__ float sg[TP][CO];
  constexpr int BG = 256 / CO;  // bias lane groups
  static_assert(256 % CO == 0, "bias groups");
  const int t = threadIdx.x;
  const int blk = t % NB, pg = t / NB;
  const int bco = t % CO, bg = t / CO;
  const int rb = blk / (CO / 4), cb = blk % (CO / 4);
  float acc[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[r][c] = 0.f;
  float bacc = 0.f;
  // 32-bit pixel indexing (B H W < 2^31, checked at drq_create): the tap's input pixel is
  // pix + dy W + dx inside the image, so only x and y need a division
  const int npix = B * H * W;
  for (int p0 = blockIdx.x * TP; p0 < npix; p0 += gridDim.x * TP) {
    __syncthreads();
    for (int pr = t; pr < TP * 9; pr += 256) {
      const int q = pr / 9, tap = pr - 9 * q;
      const int pix = p0 + q;
      float v[CI];
#pragma unroll
      for (int ci = 0; ci < CI; ++ci) v[ci] = 0.f;
      if (pix < npix) {
        const int r = pix / W;
        const int x = pix - r * W, y = r % H;
        const int dy = tap / 3 - 1, dx = tap % 3 - 1;
        const int yy = y + dy, xx = x + dx;
        if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
          const float* ip = in + (long long)(pix + dy * W + dx) * CI;
#pragma unroll
          for (int c4 = 0; c4 < CI; c4 += 4) {
            const float4 u = *reinterpret_cast<const float4*>(ip + c4);
            v[c4] = u.x; v[c4 + 1] = u.y; v[c4 + 2] = u.z; v[c4 + 3] = u.w;
          }
        }
      }
#pragma unroll
      for (int ci = 0; ci < CI; ++ci) sin_[q][tap * CI + ci] = RELU_IN ? fmaxf(v[ci], 0.f) : v[ci];
    }
    for (int pr = t; pr < TP * CO; pr += 256) {
      const int q = pr / CO, co = pr - CO * q;
      const int pix = p0 + q;
      sg[q][co] = pix < npix ? dout[(long long)pix * CO + co] : 0.f;
    }
    __syncthreads();
    if (t < NB * PG) {  // 4 x 4 register block: two ds_read_b128 feed sixteen FMAs
      const float4* ar = reinterpret_cast<const float4*>(&sin_[0][4 * rb]);
      const float4* gr = reinterpret_cast<const float4*>(&sg[0][4 * cb]);
      for (int q = pg; q < TP; q += PG) {
        const float4 a = ar[q * (9 * CI / 4)];
        const float4 g = gr[q * (CO / 4)];
        const float av[4] = {a.x, a.y, a.z, a.w}, gv[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int c = 0; c < 4; ++c) acc[r][c] = fmaf(av[r], gv[c], acc[r][c]);
      }
    }
    {  // bias: lane group bg sums pixels q = bg, bg + BG, ... of channel bco (all lanes busy)
      float s = bacc;
      for (int q = bg; q < TP; q += BG) s += sg[q][bco];
      bacc = s;
    }
  }
  // the PG pixel-group partials of each block, summed in group order
  __shared__ float red[PG > 1 ? NB * PG * 16 : 1];
  float* pp = part + (long long)blockIdx.x * (NW + CO);
  if (PG > 1) {
    __syncthreads();
    if (t < NB * PG)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) red[(pg * NB + blk) * 16 + r * 4 + c] = acc[r][c];
    __syncthreads();
    if (t < NB) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        float v = red[blk * 16 + e];
        for (int g = 1; g < PG; ++g) v += red[(g * NB + blk) * 16 + e];
        acc[e >> 2][e & 3] = v;
      }
    }
  }
  if (t < NB)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      *reinterpret_cast<float4*>(pp + (4 * rb + r) * CO + 4 * cb) =
          make_float4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
  // the bias groups' partials, summed in group order
  __shared__ float bred[256];
  __syncthreads();
  bred[t] = bacc;
  __syncthreads();
  if (t < CO) {
    float v = bred[t];
    for (int g = 1; g < BG; ++g) v += bred[g * CO + t];
    pp[NW + t] = v;
  }
}

// Weight gradient partials on row tiles (round 6, the default; conv_wgrad_kernel above is the
// im2col form it replaced).  A tile is R consecutive rows of one image; its R + 2 input rows (act
// applied, one zero column each side, zero outside the image) and its R dout rows are staged in LDS
// ONCE, and the nine taps read the padded rows at shifted offsets, so the staging moves (R + 2) / R
// copies of the input instead of im2col's nine, with no per-row index arithmetic (the per-slot
// offsets are the same for every tile and computed once).  Lane (pg, blk): blk = (tap, block of CB
// input channels) owns a CB x CO block of dW -- 8 x 16 FMAs per two plus four ds_read_b128, so
// the loop is VALU-bound, not LDS-bound as the 4 x 4 blocks above were -- over the pixels q = pg,
// pg + PG, ... of every tile; the next tile is loaded into registers (unconditionally, at a clamped
// address) while this one is computed.  The PG groups' partials are added in a fixed tree order
// in LDS and the bias sums as in conv_wgrad_kernel, so the result is reproducible run to run.
// part[g][9 CI CO + CO] as conv_wgrad_kernel.
template <int CI, int CO>
struct WgRows {
  static constexpr int CB = CI < 8 ? CI : 8;  // input channels per lane block
  static constexpr int NB = 9 * (CI / CB);    // lane blocks (each: one tap, CB channels, all CO)
  static constexpr int PG = 256 / NB;         // pixel groups
  static constexpr int NPF = 8;               // staged float4 per thread per tile
  static constexpr int E4 = CB * CO / 4;      // float4 of one lane's block
  static constexpr int RED4 = (PG / 2) * NB * E4;
  static constexpr int LDS4 = RED4 > NPF * 256 ? RED4 : NPF * 256;
};

template <int CI, int CO, bool RELU_IN>
__global__ __launch_bounds__(256) void conv_wgrad_rows_kernel(const float* __restrict__ in, const float* __restrict__ dout,
                                                              float* __restrict__ part, WgGeo geo) {
  using P = WgRows<CI, CO>;
  constexpr int CB = P::CB, NB = P::NB, PG = P::PG, NPF = P::NPF, E4 = P::E4;
  constexpr int NW = 9 * CI * CO;
  constexpr int BG = 256 / CO;
  static_assert(CI % 4 == 0 && CO % 4 == 0 && 256 % CO == 0, "channels");
  __shared__ float4 lds4[P::LDS4];
  __shared__ float bred[256];
  float* const lds = reinterpret_cast<float*>(lds4);
  const int H = geo.H, W = geo.W, R = geo.R, SR = geo.SR;
  const int NI = (R + 2) * (W + 2) * (CI / 4), NT = NI + R * W * (CO / 4);
  const int tpi = (H + R - 1) / R;
  float* const s_g = lds + (R + 2) * SR;
  const int t = threadIdx.x;
  // staging slots k: input float4 (row i, column j, chunk c) or dout float4 (row r, column x, chunk c);
  // offsets from the tile's base pixel, the row relative to the tile's first row (validity), LDS offset
  int soff[NPF], loff[NPF], rrel[NPF];
  bool isg[NPF];
#pragma unroll
  for (int k = 0; k < NPF; ++k) {
    const int s = t + 256 * k;
    isg[k] = s >= NI;
    if (s < NI) {
      const int c = s % (CI / 4), j = (s / (CI / 4)) % (W + 2), i = s / ((CI / 4) * (W + 2));
      soff[k] = ((i - 1) * W + (j - 1)) * CI + 4 * c;
      loff[k] = i * SR + j * CI + 4 * c;
      rrel[k] = (j >= 1 && j <= W) ? i - 1 : -(1 << 20);  // padding columns: never valid
    } else if (s < NT) {
      const int u = s - NI, c = u % (CO / 4), q = u / (CO / 4);
      soff[k] = q * CO + 4 * c;  // q = r W + x
      loff[k] = (R + 2) * SR + q * CO + 4 * c;
      rrel[k] = q / W;
    } else {
      soff[k] = 0;
      loff[k] = -1;
      rrel[k] = -(1 << 20);
    }
  }
  float4 v[NPF];
  auto load_tile = [&](int tile) {
    const int b = tile / tpi, y0 = (tile - b * tpi) * R;
    const long long p0 = ((long long)b * H + y0) * W;
    const float* ib = in + p0 * CI;
    const float* gb = dout + p0 * CO;
#pragma unroll
    for (int k = 0; k < NPF; ++k) {
      const bool ok = (unsigned)(y0 + rrel[k]) < (unsigned)H;
      const float* src = ok ? (isg[k] ? gb : ib) + soff[k] : ib;  // ib: row y0 of image b, always in range
      const float4 u = *reinterpret_cast<const float4*>(src);
      float4 w = ok ? u : make_float4(0.f, 0.f, 0.f, 0.f);
      if (RELU_IN && !isg[k]) w = make_float4(fmaxf(w.x, 0.f), fmaxf(w.y, 0.f), fmaxf(w.z, 0.f), fmaxf(w.w, 0.f));
      v[k] = w;
    }
  };
  const int blk = t % NB, pg = t / NB;
  const int tap = blk / (CI / CB), cb0 = (blk % (CI / CB)) * CB;
  const int aoff = (tap / 3) * SR + (tap % 3) * CI + cb0;
  const int bco = t % CO, bg = t / CO;
  float acc[CB][CO];
#pragma unroll
  for (int i = 0; i < CB; ++i)
#pragma unroll
    for (int j = 0; j < CO; ++j) acc[i][j] = 0.f;
  float bacc = 0.f;
  const int npx = R * W;
  if ((int)blockIdx.x < geo.tiles) load_tile(blockIdx.x);
  for (int tile = blockIdx.x; tile < geo.tiles; tile += gridDim.x) {
    __syncthreads();  // the previous tile's reads are done
#pragma unroll
    for (int k = 0; k < NPF; ++k)
      if (loff[k] >= 0) *reinterpret_cast<float4*>(lds + loff[k]) = v[k];
    __syncthreads();
    load_tile(min(tile + (int)gridDim.x, geo.tiles - 1));  // in flight during this tile's FMAs
    if (t < NB * PG) {
      for (int q = pg; q < npx; q += PG) {
        const int r = __umulhi((unsigned)q, geo.magic), x = q - r * W;
        const float* ap = lds + aoff + r * SR + x * CI;
        const float* gp = s_g + q * CO;
        float a[CB], g[CO];
#pragma unroll
        for (int c4 = 0; c4 < CB; c4 += 4) {
          const float4 u = *reinterpret_cast<const float4*>(ap + c4);
          a[c4] = u.x; a[c4 + 1] = u.y; a[c4 + 2] = u.z; a[c4 + 3] = u.w;
        }
#pragma unroll
        for (int c4 = 0; c4 < CO; c4 += 4) {
          const float4 u = *reinterpret_cast<const float4*>(gp + c4);
          g[c4] = u.x; g[c4 + 1] = u.y; g[c4 + 2] = u.z; g[c4 + 3] = u.w;
        }
#pragma unroll
        for (int i = 0; i < CB; ++i)
#pragma unroll
          for (int j = 0; j < CO; ++j) acc[i][j] = fmaf(a[i], g[j], acc[i][j]);
      }
    }
    {  // bias: lane group bg sums pixels q = bg, bg + BG, ... of channel bco (rows past H are zero)
      float s = bacc;
      for (int q = bg; q < npx; q += BG) s += s_g[q * CO + bco];
      bacc = s;
    }
  }
  // the PG groups' partials, added in a fixed tree order (group pg + s into group pg)
  float4* const red = lds4;
#pragma unroll 1
  for (int s = 1; s < PG; s *= 2) {
    __syncthreads();
    if (t < NB * PG && pg % (2 * s) == s) {
      float4* d = red + (pg / (2 * s)) * E4 * NB + blk;
#pragma unroll
      for (int e = 0; e < E4; ++e) {
        const int i = (4 * e) / CO, j = (4 * e) % CO;
        d[e * NB] = make_float4(acc[i][j], acc[i][j + 1], acc[i][j + 2], acc[i][j + 3]);
      }
    }
    __syncthreads();
    if (t < NB * PG && pg % (2 * s) == 0 && pg + s < PG) {
      const float4* d = red + (pg / (2 * s)) * E4 * NB + blk;
#pragma unroll
      for (int e = 0; e < E4; ++e) {
        const int i = (4 * e) / CO, j = (4 * e) % CO;
        const float4 u = d[e * NB];
        acc[i][j] += u.x; acc[i][j + 1] += u.y; acc[i][j + 2] += u.z; acc[i][j + 3] += u.w;
      }
    }
  }
  float* pp = part + (long long)blockIdx.x * (NW + CO);
  if (t < NB)
#pragma unroll
    for (int i = 0; i < CB; ++i)
#pragma unroll
      for (int j = 0; j < CO; j += 4)
        *reinterpret_cast<float4*>(pp + (tap * CI + cb0 + i) * CO + j) =
            make_float4(acc[i][j], acc[i][j + 1], acc[i][j + 2], acc[i][j + 3]);
  __syncthreads();
  bred[t] = bacc;
  __syncthreads();
  if (t < CO) {
    float s = bred[t];
    for (int g = 1; g < BG; ++g) s += bred[g * CO + t];
    pp[NW + t] = s;
  }
}

// Forward and data-gradient convolutions on row tiles (round 6).  One block = one tile of R rows of
// one image; its R + 2 input rows (zero-padded by one column each side and zero outside the image;
// act applied) are staged in LDS once, and every lane reads its pixel's nine neighbours from there
// instead of from L1 (the one-lane-per-pixel kernels above read each input pixel nine times through
// the texture path, which bounds them next to the FMAs).  Weights stay wave-uniform scalar loads:
// wave w computes the CG output channels of group w % NG for pixels (w / NG) 64 + lane of the tile.
//   FWD:  out[p][o] = bias[o] + sum_{tap,k} act(X)[p + off(tap)][k] w[tap][k][o]  (+ res[p][o]),
//         X = the conv input (KI = ci, KO = co); images [0, B1) take (w_a, bias_a), the rest (w_b, bias_b)
//   !FWD: din[p][j] = (sum_{tap,k} dout[p + off(tap)][k] w[8 - tap][j][k]) [mask[p][j] > 0] (+ dres[p][j]),
//         X = dout (KI = co, KO = ci): the transposed conv as a conv with the taps flipped.
// The per-output summation order (taps, then input channels) is that of the kernels above; a tap
// outside the image adds fma(0, w, acc) = acc, so the results are theirs.  LDS: a pixel's KI / 4
// 16-byte chunks are stored XOR-swizzled by column (chunk c of padded column j at
// c ^ ((j / (64 / KI)) % (KI / 4))), so 16 lanes on consecutive pixels read 16 distinct bank quads.
// floats of the staged rows (16 KB; at 12 KB the 16-channel data grad at 42 x 42 got 2-row tiles).  Two
// output pixels a lane (each scalar weight feeding two FMAs) measured 2-3x slower: the compiler spilled
// the weights through VGPR lanes (profiles/r6n_drq_two_pixels_per_lane)
constexpr int CR_LDS = 4096;
template <int KI, int KO, int CG, bool FWD, bool RELU_IN, bool MASK, bool ADD_RES>
__global__ __launch_bounds__(256) void conv_rows_kernel(const float* __restrict__ X, const float* __restrict__ w_a,
                                                        const float* __restrict__ bias_a, const float* __restrict__ w_b,
                                                        const float* __restrict__ bias_b, int B1,
                                                        const float* __restrict__ mask, const float* __restrict__ res,
                                                        float* __restrict__ out, ConvGeo geo) {
  constexpr int NG = KO / CG, KC = KI / 4, PPR = 64 / KI;  // groups, chunks per pixel, pixels per 256 B
  static_assert(KO % CG == 0 && CG % 4 == 0 && KI % 4 == 0 && NG <= 4, "channels");
  __shared__ float4 lds4[CR_LDS / 4];
  float* const lds = reinterpret_cast<float*>(lds4);
  const int H = geo.H, W = geo.W, R = geo.R, SR = geo.SR;
  const int b = (int)blockIdx.x / geo.n, y0 = ((int)blockIdx.x - b * geo.n) * R;
  const long long p0 = ((long long)b * H + y0) * W;  // the tile's first pixel
  const int t = threadIdx.x;
  {  // stage rows y0 - 1 .. y0 + R: slot s = (row i, padded column j, chunk c)
    const int NS = (R + 2) * (W + 2) * KC;
    const float* base = X + p0 * KI;
#pragma unroll
    for (int k = 0; k < CR_LDS / 4 / 256; ++k) {
      const int s = t + 256 * k;
      const int c = s % KC, u = s / KC;
      const int i = __umulhi((unsigned)u, geo.magic2), j = u - i * (W + 2);
      const int yy = y0 + i - 1, xx = j - 1;
      const bool ok = s < NS && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
      const float* src = ok ? base + ((long long)(i - 1) * W + xx) * KI + 4 * c : base;
      const float4 q = *reinterpret_cast<const float4*>(src);
      float4 v = ok ? q : make_float4(0.f, 0.f, 0.f, 0.f);
      if (RELU_IN) v = make_float4(fmaxf(v.x, 0.f), fmaxf(v.y, 0.f), fmaxf(v.z, 0.f), fmaxf(v.w, 0.f));
      if (s < NS) *reinterpret_cast<float4*>(lds + i * SR + j * KI + 4 * (c ^ ((j / PPR) % KC))) = v;
    }
  }
  __syncthreads();
  const int wv = __builtin_amdgcn_readfirstlane(t >> 6), g = wv % NG;  // wave-uniform: scalar weight loads
  const int q = (wv / NG) * 64 + (t & 63);
  const int r = __umulhi((unsigned)q, geo.magic), x = q - r * W;
  if (q >= R * W || y0 + r >= H) return;  // no barrier follows
  const float* __restrict__ w = (FWD && b >= B1) ? w_b : w_a;
  float acc[CG];
#pragma unroll
  for (int c = 0; c < CG; ++c) acc[c] = FWD ? ((b >= B1) ? bias_b : bias_a)[g * CG + c] : 0.f;
#pragma unroll
  for (int tt = 0; tt < 9; ++tt) {  // !FWD: X tap 8 - tt is weight tap tt, in the order above
    const int tap = FWD ? tt : 8 - tt;
    const int j = x + tap % 3;
    const float* xp = lds + (r + tap / 3) * SR + j * KI;
    const int sw = (j / PPR) % KC;
    float v[KI];
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      const float4 u = *reinterpret_cast<const float4*>(xp + 4 * (c ^ sw));
      v[4 * c] = u.x; v[4 * c + 1] = u.y; v[4 * c + 2] = u.z; v[4 * c + 3] = u.w;
    }
#pragma unroll
    for (int k = 0; k < KI; ++k) {
#pragma unroll
      for (int c = 0; c < CG; ++c) {
        const float wk = FWD ? w[(tap * KI + k) * KO + g * CG + c] : w[(tt * KO + g * CG + c) * KI + k];
        acc[c] = fmaf(v[k], wk, acc[c]);
      }
    }
  }
  const long long o = (p0 + (long long)r * W + x) * KO + g * CG;
#pragma unroll
  for (int c4 = 0; c4 < CG; c4 += 4) {
    float4 v = make_float4(acc[c4], acc[c4 + 1], acc[c4 + 2], acc[c4 + 3]);
    if (MASK) {
      const float4 m = *reinterpret_cast<const float4*>(mask + o + c4);
      v.x = m.x > 0.f ? v.x : 0.f; v.y = m.y > 0.f ? v.y : 0.f;
      v.z = m.z > 0.f ? v.z : 0.f; v.w = m.w > 0.f ? v.w : 0.f;
    }
    if (ADD_RES) {
      const float4 a = *reinterpret_cast<const float4*>(res + o + c4);
      v.x += a.x; v.y += a.y; v.z += a.z; v.w += a.w;
    }
    *reinterpret_cast<float4*>(out + o + c4) = v;
  }
}

// ------------------------------------------------------------------ convolutions on split2h MFMA
// Forward and data gradient of the 8- and 16-channel convs as implicit GEMMs on v_mfma_f32_16x16x32_f16
// with the split2h planes of the SAC path (gemm_common.h: x 2^e = h + l in fp16, products h l, l h, h h,
// fp32 accumulation; the dropped l l is <= 2^-22 relative).  One block = one row tile (conv_rows_kernel's
// geometry); its R + 2 input rows are loaded, their max |x| taken over the block and the tile's
// exponent chosen from it, then split ONCE into two fp16 planes in LDS ([plane][row][column][channel],
// zero-padded) -- the nine taps read the planes at shifted offsets, so nothing is split twice.  The
// weights' exponent comes from their max |w| (each block reads all of them) and every lane holds
// its B fragments (k-slices of 32 = taps x channels, N = 16 output channels, zero past 9 KI and KO)
// split in registers for the whole block.  A lane's A fragment of M-tile m, slice s: pixel 16 m +
// (lane & 15), k = 32 s + 8 (lane >> 4) .. + 7 = 8 channels of one tap (one ds_read_b128 a plane).
// The accumulator is unscaled exactly (2^-(ea + ew)) before the bias / residual (FWD) or the ReLU
// mask / residual gradient (!FWD) is applied.  FWD: X = act(in), KI = ci, KO = co, w[tap][k][n];
// !FWD: X = dout, KI = co, KO = ci, w[8 - tap][n][k] (the transposed conv).  Not bitwise the VALU
// kernels (another summation order); held to the float64 oracle like them.
typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
typedef float h2acc_t __attribute__((ext_vector_type(4)));
constexpr int CH_LDS = 6144;   // fp16 elements of one staged plane
constexpr int CH_SLOTS = 6;    // staged float4 per thread
__device__ inline int h2_exp(float bound) {  // gemm_common.h plane_exp: |x| 2^e < 2^15
  bound *= 1.00390625f;
  if (!(bound > 0.f) || !(bound < 3.0e38f)) return 0;
  int ex;
  (void)frexpf(bound, &ex);
  return min(100, max(-100, 15 - ex));
}
__device__ inline void h2_split(float x, float sc, _Float16& h, _Float16& l) {
  const float y = x * sc;
  h = (_Float16)y;
  l = (_Float16)(y - (float)h);
}
template <int KI, int KO, bool FWD, bool RELU_IN, bool MASK, bool ADD_RES>
__global__ __launch_bounds__(256) void conv_h2_kernel(const float* __restrict__ X, const float* __restrict__ w_a,
                                                      const float* __restrict__ bias_a, const float* __restrict__ w_b,
                                                      const float* __restrict__ bias_b, int B1,
                                                      const float* __restrict__ mask, const float* __restrict__ res,
                                                      float* __restrict__ out, ConvGeo geo) {
  static_assert(KI == 8 || KI == 16, "input channels");
  static_assert(KO == 4 || KO == 8 || KO == 16, "output channels");
  constexpr int NS = (9 * KI + 31) / 32;  // k-slices
  __shared__ __attribute__((aligned(16))) _Float16 sh[2][CH_LDS];
  __shared__ float red[2][4];
  const int H = geo.H, W = geo.W, R = geo.R, WP = W + 2;
  const int b = (int)blockIdx.x / geo.n, y0 = ((int)blockIdx.x - b * geo.n) * R;
  const long long p0 = ((long long)b * H + y0) * W;
  const float* __restrict__ w = (FWD && b >= B1) ? w_b : w_a;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  // 1. the tile's rows y0 - 1 .. y0 + R into registers (zero outside the image), their max |x|
  const int NSL = (R + 2) * WP * (KI / 4);
  const float* base = X + p0 * KI;
  float4 v[CH_SLOTS];
  int lo[CH_SLOTS];
  float mx = 0.f, mw = 0.f;
#pragma unroll
  for (int k = 0; k < CH_SLOTS; ++k) {
    const int s = t + 256 * k;
    const int c = s % (KI / 4), u = s / (KI / 4);
    const int i = __umulhi((unsigned)u, geo.magic2), j = u - i * WP;
    const int yy = y0 + i - 1, xx = j - 1;
    const bool ok = s < NSL && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
    const float4 q = *reinterpret_cast<const float4*>(ok ? base + ((long long)(i - 1) * W + xx) * KI + 4 * c : base);
    float4 x4 = ok ? q : make_float4(0.f, 0.f, 0.f, 0.f);
    if (RELU_IN) x4 = make_float4(fmaxf(x4.x, 0.f), fmaxf(x4.y, 0.f), fmaxf(x4.z, 0.f), fmaxf(x4.w, 0.f));
    v[k] = x4;
    lo[k] = s < NSL ? (i * WP + j) * KI + 4 * c : -1;
    mx = fmaxf(mx, fmaxf(fmaxf(fabsf(x4.x), fabsf(x4.y)), fmaxf(fabsf(x4.z), fabsf(x4.w))));
  }
#pragma unroll
  for (int e0 = 0; e0 < 9 * KI * KO; e0 += 256) {  // unrolled: the weight loads in flight together
    const int e = min(e0 + t, 9 * KI * KO - 1);
    mw = fmaxf(mw, fabsf(w[e]));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mx = fmaxf(mx, __shfl_xor(mx, o));
    mw = fmaxf(mw, __shfl_xor(mw, o));
  }
  if (lane == 0) {
    red[0][wv] = mx;
    red[1][wv] = mw;
  }
  __syncthreads();
  mx = fmaxf(fmaxf(red[0][0], red[0][1]), fmaxf(red[0][2], red[0][3]));
  mw = fmaxf(fmaxf(red[1][0], red[1][1]), fmaxf(red[1][2], red[1][3]));
  const int ea = h2_exp(mx), ew = h2_exp(mw);
  const float sa = ldexpf(1.f, ea), sw = ldexpf(1.f, ew), unscale = ldexpf(1.f, -(ea + ew));
  // 2. split once into the LDS planes
#pragma unroll
  for (int k = 0; k < CH_SLOTS; ++k) {
    if (lo[k] < 0) continue;
    _Float16 h0, l0, h1, l1, h2, l2, h3, l3;
    h2_split(v[k].x, sa, h0, l0);
    h2_split(v[k].y, sa, h1, l1);
    h2_split(v[k].z, sa, h2, l2);
    h2_split(v[k].w, sa, h3, l3);
    typedef _Float16 h4_t __attribute__((ext_vector_type(4)));
    *reinterpret_cast<h4_t*>(&sh[0][lo[k]]) = h4_t{h0, h1, h2, h3};
    *reinterpret_cast<h4_t*>(&sh[1][lo[k]]) = h4_t{l0, l1, l2, l3};
  }
  // 3. the B fragments: lane holds B[k = 32 s + 8 (lane >> 4) + e][n = lane & 15], e < 8
  const int n = lane & 15, kq = 8 * (lane >> 4);
  h8_t bh[NS], bl[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = 32 * s + kq + e, tap = k / KI, c = k % KI;
      float wk = 0.f;
      if (k < 9 * KI && n < KO) wk = FWD ? w[(tap * KI + c) * KO + n] : w[((8 - tap) * KO + n) * KI + c];
      _Float16 hh, ll;
      h2_split(wk, sw, hh, ll);
      bh[s][e] = hh;
      bl[s][e] = ll;
    }
  }
  __syncthreads();
  // 4. 16-pixel M-tiles, round robin over the waves
  const int npx = R * W, nmt = (npx + 15) / 16;
  for (int mt = wv; mt < nmt; mt += 4) {
    const int q = min(16 * mt + (lane & 15), npx - 1);
    const int r = __umulhi((unsigned)q, geo.magic), x = q - r * W;
    h2acc_t acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int kb = 32 * s + kq;
      const int tap = min(kb / KI, 8), c0 = kb % KI;  // tap 9..: zero weights, any finite A
      const int off = ((r + tap / 3) * WP + x + tap % 3) * KI + c0;
      const h8_t ah = *reinterpret_cast<const h8_t*>(&sh[0][off]);
      const h8_t al = *reinterpret_cast<const h8_t*>(&sh[1][off]);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[s], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[s], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[s], acc, 0, 0, 0);
    }
    // lane holds C[pixel 16 mt + 4 (lane >> 4) + i][channel lane & 15]
    if (n < KO) {
      const float bn = FWD ? ((b >= B1) ? bias_b : bias_a)[n] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int qq = 16 * mt + 4 * (lane >> 4) + i;
        if (qq >= npx) continue;
        const int rr = __umulhi((unsigned)qq, geo.magic), xx = qq - rr * W;
        if (y0 + rr >= H) continue;
        const long long o = (p0 + (long long)rr * W + xx) * KO + n;
        float val = acc[i] * unscale + bn;
        if (MASK && !(mask[o] > 0.f)) val = 0.f;
        if (ADD_RES) val += res[o];
        out[o] = val;
      }
    }
  }
}

// ------------------------------------------------------------------ convolutions on f32 MFMA
// v_mfma_f32_16x16x4_f32 (exact fp32: bit for bit a k-ordered fmaf chain, MI355X_MICROARCH.md) at the
// FP32 rate, which the VALU kernels above reach only with packed FMAs fed from SGPRs; here the VALU
// only computes addresses and the operands come straight from L1/L2 one fp32 per lane.
typedef float f32x4_t __attribute__((ext_vector_type(4)));

// Weight gradient as 9 / TPM small GEMMs over pixels: dW[tap][ci][co] = sum_p act(in)[p + off(tap)][ci]
// * dout[p][co].  M-tile m stacks TPM = 16 / CI taps (rows r: tap m TPM + r / CI, channel r % CI), N = CO
// (columns >= CO zero), K = pixels, 4 per MFMA (lane slot l >> 4).  A lane's A operand is one input
// channel of one shifted pixel (16 lanes read 16 consecutive floats), its B operand dout[p][l & 15],
// shared by every M-tile.  Every load is unconditional (a clamped in-range address, the value selected
// afterwards): a load under a branch was waited for at the branch's end, one latency per operand.
// Wave w of a block takes pixels c0 + 16 j + 4 w + slot of the block's chunk; each fp32 MFMA chain runs
// FLUSH k-steps and is then added into double accumulators (the bias sum is double throughout); the four
// waves' sums are added in wave order in LDS.  part[g][9 CI CO + CO] as conv_wgrad_kernel.
template <int CI, int CO, bool RELU_IN>
__global__ __launch_bounds__(256) void conv_wgrad_mfma_kernel(const float* __restrict__ in, const float* __restrict__ dout,
                                                              float* __restrict__ part, int B, int H, int W, int chunk) {
  constexpr int TPM = 16 / CI, MT = (9 + TPM - 1) / TPM;
  constexpr int NW = 9 * CI * CO;
  constexpr int FLUSH = 32;
  static_assert(CI == 4 || CI == 8 || CI == 16, "CI");
  static_assert(CO == 8 || CO == 16, "CO");
  __shared__ double red[MT * 256];
  __shared__ double bred[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int row = lane & 15, slot = lane >> 4;
  const int ci = row % CI, tsub = row / CI;
  const int npix = B * H * W;
  const int c0 = blockIdx.x * chunk, c1 = min(npix, c0 + chunk);
  int dys[MT], dxs[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int tap = m * TPM + tsub;
    dys[m] = tap < 9 ? tap / 3 - 1 : 99;
    dxs[m] = tap < 9 ? tap % 3 - 1 : 0;
  }
  double accd[MT][4];
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int r = 0; r < 4; ++r) accd[m][r] = 0.0;
  double bsum = 0.0;
  const bool gcol = row < CO;
  int p = c0 + 4 * wv + slot;
  int x = p % W, y = (p / W) % H;
  const int nsteps = c1 > c0 ? (c1 - c0 + 15) / 16 : 0;
  // operands of one k-step (this lane's pixel p at (x, y)), loaded one k-step ahead of its MFMAs
  float av[MT], g = 0.f;
  auto load = [&](int pp, int xx0, int yy0, float* a, float& gg) {
    const bool vp = pp < c1;
    const int pc = vp ? pp : c0;  // an in-range pixel for the unconditional loads
    const float gl = dout[(long long)pc * CO + (gcol ? row : 0)];
    gg = (vp && gcol) ? gl : 0.f;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int yy = yy0 + dys[m], xx = xx0 + dxs[m];
      const bool ok = vp && yy >= 0 && yy < H && xx >= 0 && xx < W;
      const int q = ok ? pp + dys[m] * W + dxs[m] : pc;
      const float v = in[(long long)q * CI + ci];
      a[m] = ok ? (RELU_IN ? fmaxf(v, 0.f) : v) : 0.f;
    }
  };
  auto advance = [&]() {  // this lane's next pixel: 16 on (W >= 4: at most 4 wraps)
    p += 16;
    x += 16;
    while (x >= W) {
      x -= W;
      if (++y == H) y = 0;
    }
  };
  if (nsteps > 0) load(p, x, y, av, g);
  for (int s0 = 0; s0 < nsteps; s0 += FLUSH) {
    f32x4_t acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const int s1 = min(nsteps, s0 + FLUSH);
    for (int s = s0; s < s1; ++s) {
      advance();
      float an[MT], gn = 0.f;
      if (s + 1 < nsteps) load(p, x, y, an, gn);  // uniform: the whole wave takes it
      bsum += (double)g;
#pragma unroll
      for (int m = 0; m < MT; ++m) acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[m], g, acc[m], 0, 0, 0);
#pragma unroll
      for (int m = 0; m < MT; ++m) av[m] = an[m];
      g = gn;
    }
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) accd[m][r] += (double)acc[m][r];
  }
  // C layout: register r of lane l = row 4 (l >> 4) + r of the tile, column l & 15; waves in order
  for (int w = 0; w < 4; ++w) {
    if (wv == w)
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int e = m * 256 + (4 * slot + r) * 16 + row;
          red[e] = w == 0 ? accd[m][r] : red[e] + accd[m][r];
        }
    __syncthreads();
  }
  bred[wv][lane] = bsum;
  __syncthreads();
  float* pp = part + (long long)blockIdx.x * (NW + CO);
  for (int e = threadIdx.x; e < MT * 256; e += 256) {
    const int m = e >> 8, rr = (e >> 4) & 15, cc = e & 15;
    const int tap = m * TPM + rr / CI;
    if (tap >= 9 || cc >= CO) continue;
    pp[(tap * CI + rr % CI) * CO + cc] = (float)red[e];
  }
  if (threadIdx.x < CO) {
    double v = 0.0;
#pragma unroll
    for (int w = 0; w < 4; ++w)
#pragma unroll
      for (int s = 0; s < 4; ++s) v += bred[w][16 * s + threadIdx.x];
    pp[NW + threadIdx.x] = (float)v;
  }
}

// Forward (FWD) and data gradient (!FWD) as pixel-tile GEMMs: out[p][n] = sum_{tap, c} X[p + off][c] *
// Wk[tap][c][n], K = 9 KC, N = NC.  FWD: X = act(in), KC = CI, NC = CO, off = +tap, Wk = w, C starts at
// the bias, + res.  !FWD: X = dout, KC = CO, NC = CI, off = -tap, Wk[tap][c][n] = w[tap][n][c], C starts
// at 0, * [mask > 0] + dres.  A lane loads float4s: lane group g = l >> 4 takes tap TPG-group member
// g / (KC / 4) and channels 4 (g % (KC / 4)) .. + 3, element j of them feeding k-step j (TPG = 16 / KC taps
// per load round).  The B fragments (one weight per k-step) stay in VGPRs; each wave runs TW 16-pixel
// tiles side by side (independent accumulators) over the block's 64 TW consecutive pixels.  Images
// [0, B1) use (w_a, bias_a), [B1, B) (w_b, bias_b): separate blocks, as conv_fwd_kernel.
template <int KC, int NC, bool FWD, bool RELU_IN, bool ADD_RES, int TW>
__global__ __launch_bounds__(256) void conv_mfma_kernel(const float* __restrict__ X, const float* __restrict__ w_a,
                                                        const float* __restrict__ bias_a, const float* __restrict__ w_b,
                                                        const float* __restrict__ bias_b, const float* __restrict__ mask,
                                                        const float* __restrict__ res, float* __restrict__ out, int B,
                                                        int B1, int H, int W) {
  constexpr int CG4 = KC / 4, TPG = 4 / CG4, ROUNDS = (9 + TPG - 1) / TPG, NK = ROUNDS * 4;
  constexpr int PB = 4 * 16 * TW;  // pixels per block
  static_assert(KC == 4 || KC == 8 || KC == 16, "KC");
  static_assert(NC == 4 || NC == 8 || NC == 16, "NC");
  const int n1 = B1 * H * W, nb1 = (n1 + PB - 1) / PB;
  const bool second = (int)blockIdx.x >= nb1;
  const int base = second ? n1 + ((int)blockIdx.x - nb1) * PB : (int)blockIdx.x * PB;
  const int end = second ? B * H * W : n1;
  const float* __restrict__ w = second ? w_b : w_a;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int col = lane & 15, g = lane >> 4;
  const int tg = g / CG4, c4 = 4 * (g % CG4);
  float bw[NK];
#pragma unroll
  for (int r = 0; r < ROUNDS; ++r) {
    const int tap = r * TPG + tg;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float v = 0.f;
      if (tap < 9 && col < NC) {
        const int c = c4 + j;
        v = FWD ? w[(tap * KC + c) * NC + col] : w[(tap * NC + col) * KC + c];
      }
      bw[r * 4 + j] = v;
    }
  }
  const float b0 = (FWD && col < NC) ? (second ? bias_b : bias_a)[col] : 0.f;
  f32x4_t acc[TW];
  int px[TW], xs[TW], ys[TW];
  const int p0 = base + wv * 16 * TW;
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    acc[t] = f32x4_t{b0, b0, b0, b0};
    px[t] = p0 + 16 * t + col;
    xs[t] = px[t] % W;
    ys[t] = (px[t] / W) % H;
  }
#pragma unroll
  for (int r = 0; r < ROUNDS; ++r) {
    const int tap = r * TPG + tg;
    const int dy = FWD ? tap / 3 - 1 : 1 - tap / 3, dx = FWD ? tap % 3 - 1 : 1 - tap % 3;
    float4 a[TW];
#pragma unroll
    for (int t = 0; t < TW; ++t) {  // unconditional loads from clamped addresses, values selected after
      const int yy = ys[t] + dy, xx = xs[t] + dx;
      const bool ok = tap < 9 && px[t] < end && yy >= 0 && yy < H && xx >= 0 && xx < W;
      const int q = ok ? px[t] + dy * W + dx : base;
      const float4 v = *reinterpret_cast<const float4*>(X + (long long)q * KC + c4);
      a[t].x = ok ? (RELU_IN ? fmaxf(v.x, 0.f) : v.x) : 0.f;
      a[t].y = ok ? (RELU_IN ? fmaxf(v.y, 0.f) : v.y) : 0.f;
      a[t].z = ok ? (RELU_IN ? fmaxf(v.z, 0.f) : v.z) : 0.f;
      a[t].w = ok ? (RELU_IN ? fmaxf(v.w, 0.f) : v.w) : 0.f;
    }
#pragma unroll
    for (int t = 0; t < TW; ++t) {
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t].x, bw[r * 4 + 0], acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t].y, bw[r * 4 + 1], acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t].z, bw[r * 4 + 2], acc[t], 0, 0, 0);
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t].w, bw[r * 4 + 3], acc[t], 0, 0, 0);
    }
  }
  if (col >= NC) return;
#pragma unroll
  for (int t = 0; t < TW; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int p = p0 + 16 * t + 4 * g + r;
      if (p >= end) continue;
      const long long o = (long long)p * NC + col;
      float v = acc[t][r];
      if (!FWD && mask != nullptr) v = mask[o] > 0.f ? v : 0.f;
      if (ADD_RES) v += res[o];
      out[o] = v;
    }
}

// dw[e] / db[e - nw] = sum_g part[g][e] (e < n): block of 16 entries x 16 lane groups over g
// (g = group + 16 j, 8 loads in flight), double accumulation, the groups added in order
__device__ inline void sum_parts_block(const float* __restrict__ part, int G, int n, float* __restrict__ dst_w,
                                       float* __restrict__ dst_b, int nw, int bx) {
  __shared__ double red[16][16];
  const int el = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int e = bx * 16 + el;
  double s = 0.0;
  if (e < n) {
    int g = grp;
    for (; g + 112 < G; g += 128) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(long long)(g + 16 * u) * n + e];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += (double)v[u];
    }
    for (; g < G; g += 16) s += (double)part[(long long)g * n + e];
  }
  red[grp][el] = s;
  __syncthreads();
  if (grp == 0 && e < n) {
    double t = red[0][el];
    for (int k = 1; k < 16; ++k) t += red[k][el];
    if (e < nw) dst_w[e] = (float)t;
    else dst_b[e - nw] = (float)t;
  }
}

__global__ __launch_bounds__(256) void sum_parts_kernel(const float* __restrict__ part, int G, int n,
                                                        float* __restrict__ dst_w, float* __restrict__ dst_b, int nw) {
  sum_parts_block(part, G, n, dst_w, dst_b, nw, blockIdx.x);
}

// every conv's partials of one backward in one launch: block ranges per segment (blk0 ascending)
__global__ __launch_bounds__(256) void sum_parts_multi_kernel(const SumSeg* __restrict__ segs, int nseg) {
  int k = 0;
  while (k + 1 < nseg && (int)blockIdx.x >= segs[k + 1].blk0) ++k;
  const SumSeg sg = segs[k];
  sum_parts_block(sg.part, sg.G, sg.n, sg.dw, sg.db, sg.nw, (int)blockIdx.x - sg.blk0);
}

// ------------------------------------------------------------------ max pool 3x3 / 2 / SAME
// out[b][oy][ox][c] = max over the window (lo padding, -inf outside); arg = argmax tap (0..8,
// first in row-major order on ties -- lax.reduce_window's max has no defined tie rule for the
// gradient; jax's select-and-scatter takes the first maximum, as here)
__global__ void maxpool_fwd_kernel(const float* __restrict__ in, float* __restrict__ out,
                                   unsigned char* __restrict__ arg, int B, int H, int W, int C, int Ho, int Wo, int lo) {
  // one lane per 4 channels of one output pixel: float4 loads / stores, 32-bit index math.  The nine
  // window loads are unconditional (clamped into the image, an outside tap then skipped), so they are
  // all in flight at once: under a branch each was waited for at the branch's end, one latency a tap
  const int C4 = C >> 2;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * Ho * Wo * C4) return;
  const int c = (i % C4) * 4;
  int r = i / C4;
  const int ox = r % Wo;
  r /= Wo;
  const int oy = r % Ho;
  const int b = r / Ho;
  float4 v[9];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int y = min(max(2 * oy - lo + tap / 3, 0), H - 1), x = min(max(2 * ox - lo + tap % 3, 0), W - 1);
    v[tap] = *reinterpret_cast<const float4*>(in + ((b * H + y) * W + x) * C + c);
  }
  float4 best = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
  uchar4 bi = make_uchar4(0, 0, 0, 0);
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int y = 2 * oy - lo + tap / 3, x = 2 * ox - lo + tap % 3;
    if (y < 0 || y >= H || x < 0 || x >= W) continue;
    const unsigned char t = (unsigned char)tap;
    if (v[tap].x > best.x) { best.x = v[tap].x; bi.x = t; }
    if (v[tap].y > best.y) { best.y = v[tap].y; bi.y = t; }
    if (v[tap].z > best.z) { best.z = v[tap].z; bi.z = t; }
    if (v[tap].w > best.w) { best.w = v[tap].w; bi.w = t; }
  }
  const int o = ((b * Ho + oy) * Wo + ox) * C + c;
  *reinterpret_cast<float4*>(out + o) = best;
  *reinterpret_cast<uchar4*>(arg + o) = bi;
}

// din[b][y][x][c] = sum over the windows whose argmax is (y, x) of dout (a gather: deterministic),
// one lane per 4 channels of one input pixel.  A pixel lies in at most 2 x 2 windows (stride 2,
// size 3); their four (arg, dout) pairs are loaded unconditionally at clamped addresses and added in
// window order, skipping the windows that do not cover the pixel.
__global__ void maxpool_bwd_kernel(const float* __restrict__ dout, const unsigned char* __restrict__ arg,
                                   float* __restrict__ din, int B, int H, int W, int C, int Ho, int Wo, int lo) {
  const int C4 = C >> 2;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * H * W * C4) return;
  const int c = (i % C4) * 4;
  int r = i / C4;
  const int x = r % W;
  r /= W;
  const int y = r % H;
  const int b = r / H;
  // windows o with 2 o - lo <= y <= 2 o - lo + 2, in order
  const int oy0 = y + lo - 2 <= 0 ? 0 : (y + lo - 1) / 2, oy1 = min((y + lo) / 2, Ho - 1);
  const int ox0 = x + lo - 2 <= 0 ? 0 : (x + lo - 1) / 2, ox1 = min((x + lo) / 2, Wo - 1);
  uchar4 a[2][2];
  float4 d[2][2];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const int o = ((b * Ho + min(oy0 + u, Ho - 1)) * Wo + min(ox0 + v, Wo - 1)) * C + c;
      a[u][v] = *reinterpret_cast<const uchar4*>(arg + o);
      d[u][v] = *reinterpret_cast<const float4*>(dout + o);
    }
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int oy = oy0 + u, ty = y - (2 * oy - lo);
    if (oy > oy1 || ty < 0 || ty > 2) continue;
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const int ox = ox0 + v, tx = x - (2 * ox - lo);
      if (ox > ox1 || tx < 0 || tx > 2) continue;
      const unsigned char t = (unsigned char)(ty * 3 + tx);
      if (a[u][v].x == t) s.x += d[u][v].x;
      if (a[u][v].y == t) s.y += d[u][v].y;
      if (a[u][v].z == t) s.z += d[u][v].z;
      if (a[u][v].w == t) s.w += d[u][v].w;
    }
  }
  *reinterpret_cast<float4*>(din + ((b * H + y) * W + x) * C + c) = s;
}

// ------------------------------------------------------------------ encoder output + embedding
// feat[b] = [relu(enc[b]) (NHWC flatten) | emb[task_b] / (|emb| + 1e-8)], row stride ldf
__global__ void concat_kernel(const float* __restrict__ enc, int nenc, const float* __restrict__ emb, int D,
                              const int* __restrict__ task, int r0, int tmod, float* __restrict__ feat, int ldf, int B) {
  const int b = blockIdx.x;
  if (b >= B) return;
  for (int i = threadIdx.x; i < nenc; i += blockDim.x) feat[(long long)b * ldf + i] = fmaxf(enc[(long long)b * nenc + i], 0.f);
  if (threadIdx.x < 64) {
    const int t = task[(r0 + b) % tmod];
    float s = 0.f;
    for (int d = threadIdx.x; d < D; d += 64) s += emb[t * D + d] * emb[t * D + d];
    s = wsum(s);
    const float nrm = sqrtf(s) + 1e-8f;
    for (int d = threadIdx.x; d < D; d += 64) feat[(long long)b * ldf + nenc + d] = emb[t * D + d] / nrm;
  }
}

// ------------------------------------------------------------------ LayerNorm (flax, fast variance)
// y = (x + xb - mu) rstd scale + bias over F columns (xb: the preceding Dense bias, may be null);
// saves xhat (normalised) and rstd for the backward; RELU: y = max(y, 0).  One wave per row.
template <bool RELU>
__global__ void ln_fwd_kernel(const float* __restrict__ x, const float* __restrict__ xb, int ldx, int F,
                              const float* __restrict__ scale, const float* __restrict__ bias, float eps,
                              float* __restrict__ y, int ldy, float* __restrict__ xhat, float* __restrict__ rstd,
                              int B) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= B) return;
  const float* xr = x + (long long)row * ldx;
  float s = 0.f, s2 = 0.f;
  // unrolled: eight iterations' loads in flight (rolled, each was waited for before the next issued);
  // the sums keep their order
#pragma unroll 8
  for (int i = lane; i < F; i += 64) {
    const float v = xr[i] + (xb ? xb[i] : 0.f);
    s += v;
    s2 += v * v;
  }
  s = wsum(s);
  s2 = wsum(s2);
  const float mu = s / (float)F;
  const float var = fmaxf(s2 / (float)F - mu * mu, 0.f);
  const float r = 1.0f / sqrtf(var + eps);
#pragma unroll 8
  for (int i = lane; i < F; i += 64) {
    const float v = xr[i] + (xb ? xb[i] : 0.f);
    const float h = (v - mu) * r;
    xhat[(long long)row * F + i] = h;
    const float o = h * scale[i] + bias[i];
    y[(long long)row * ldy + i] = RELU ? fmaxf(o, 0.f) : o;
  }
  if (lane == 0) rstd[row] = r;
}

// dx = rstd (g - mean(g) - xhat mean(g xhat)), g = dy scale (dy masked by y > 0 when RELU).
// Column partials of dscale = sum dy xhat and dbias = sum dy per block of 4 rows: part[blk][2F].
template <bool RELU>
__global__ void ln_bwd_kernel(const float* __restrict__ dy, int lddy, const float* __restrict__ y, int ldy,
                              const float* __restrict__ xhat, const float* __restrict__ rstd,
                              const float* __restrict__ scale, int F, float* __restrict__ dx, int lddx, int B) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= B) return;
  float sg = 0.f, sgx = 0.f;
#pragma unroll 8
  for (int i = lane; i < F; i += 64) {
    float d = dy[(long long)row * lddy + i];
    if (RELU && !(y[(long long)row * ldy + i] > 0.f)) d = 0.f;
    const float g = d * scale[i];
    sg += g;
    sgx += g * xhat[(long long)row * F + i];
  }
  sg = wsum(sg) / (float)F;
  sgx = wsum(sgx) / (float)F;
  const float r = rstd[row];
#pragma unroll 8
  for (int i = lane; i < F; i += 64) {
    float d = dy[(long long)row * lddy + i];
    if (RELU && !(y[(long long)row * ldy + i] > 0.f)) d = 0.f;
    const float g = d * scale[i];
    dx[(long long)row * lddx + i] = r * (g - sg - xhat[(long long)row * F + i] * sgx);
  }
}

// dscale[i] = sum_b dy xhat, dbias[i] = sum_b dy (masked like ln_bwd): block of 16 columns x 16 row
// groups (rows g, g + 16, ...), the groups added in order
template <bool RELU>
__global__ __launch_bounds__(256) void ln_param_grad_kernel(const float* __restrict__ dy, int lddy,
                                                            const float* __restrict__ y, int ldy,
                                                            const float* __restrict__ xhat, int F, int B,
                                                            float* __restrict__ dscale, float* __restrict__ dbias) {
  // 16 columns x 16 row groups a block (F / 16 blocks: with 64 columns a block the launch had F / 64
  // = 8 blocks at F = 512), the groups' partials added in group order
  __shared__ float red[2][16][16];
  const int cl = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int i = blockIdx.x * 16 + cl;
  float a = 0.f, c = 0.f;
  if (i < F) {
    auto row = [&](int b) {
      float d = dy[(long long)b * lddy + i];
      if (RELU && !(y[(long long)b * ldy + i] > 0.f)) d = 0.f;
      a += d * xhat[(long long)b * F + i];
      c += d;
    };
    if constexpr (RELU) {  // measured: unrolled, this form got slower (7.2 -> 11.7 us), the other faster
      for (int b = grp; b < B; b += 16) row(b);
    } else {
#pragma unroll 8
      for (int b = grp; b < B; b += 16) row(b);
    }
  }
  red[0][grp][cl] = a;
  red[1][grp][cl] = c;
  __syncthreads();
  if (grp == 0 && i < F) {
    float sa = red[0][0][cl], sc = red[1][0][cl];
    for (int g = 1; g < 16; ++g) {
      sa += red[0][g][cl];
      sc += red[1][g][cl];
    }
    dscale[i] = sa;
    dbias[i] = sc;
  }
}

// column sums (the Dense_0 bias grad) of x[B][ld] over F columns, 16 row groups added in order
__global__ __launch_bounds__(256) void colsum_rows_kernel(const float* __restrict__ x, int ld, int F, int B,
                                                          float* __restrict__ out) {
  __shared__ float red[16][16];
  const int cl = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int i = blockIdx.x * 16 + cl;
  float s = 0.f;
  if (i < F)
#pragma unroll 8
    for (int b = grp; b < B; b += 16) s += x[(long long)b * ld + i];
  red[grp][cl] = s;
  __syncthreads();
  if (grp == 0 && i < F) {
    float v = red[0][cl];
    for (int g = 1; g < 16; ++g) v += red[g][cl];
    out[i] = v;
  }
}

// ------------------------------------------------------------------ dueling head + C51
// logits[b][a][z] = (val[b][z] + bv[z]) + (adv[b][a z] + ba[a z]) - mean_a(adv + ba)[z]
// from the combined head output hc[b][ldh] = [adv (A Z) | val (Z)] (bias hb likewise)
__device__ inline float head_logit(const float* hc, const float* hb, int A, int Z, int a, int z, float madv) {
  return (hc[A * Z + z] + hb[A * Z + z]) + ((hc[a * Z + z] + hb[a * Z + z]) - madv);
}

// One wave per sample: online logits at s' -> greedy a*, target distribution at a*, projected onto
// the support (drqeps.py:273-298); m[b][Z].  NZ: atoms per lane (Z <= 64 * NZ).
__global__ void c51_target_kernel(const float* __restrict__ hc_on, const float* __restrict__ hc_tg, int ldh,
                                  const float* __restrict__ hb_on, const float* __restrict__ hb_tg, int A, int Z,
                                  const float* __restrict__ rew, const float* __restrict__ done, float gamma_n,
                                  float vmin, float vmax, float* __restrict__ m, int* __restrict__ a_next, int B) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (b >= B) return;
  const float* on = hc_on + (long long)b * ldh;
  const float* tg = hc_tg + (long long)b * ldh;
  const bool zl = lane < Z;
  const float dz = (vmax - vmin) / (float)(Z - 1);
  const float sup = vmin + dz * (float)lane;  // jnp.linspace: start + step * i
  // mean over actions of the advantage (per atom), online and target
  float mon = 0.f, mtg = 0.f;
  if (zl) {
#pragma unroll 6
    for (int a = 0; a < A; ++a) {  // unrolled: the loads of six actions in flight, sums in order
      mon += on[a * Z + lane] + hb_on[a * Z + lane];
      mtg += tg[a * Z + lane] + hb_tg[a * Z + lane];
    }
    mon /= (float)A;
    mtg /= (float)A;
  }
  float bestq = -INFINITY;
  int besta = 0;
#pragma unroll 6
  for (int a = 0; a < A; ++a) {
    const float l = zl ? head_logit(on, hb_on, A, Z, a, lane, mon) : -INFINITY;
    const float mx = wmax(l);
    const float e = zl ? expf(l - mx) : 0.f;
    const float se = wsum(e);
    const float q = wsum(zl ? (e / se) * sup : 0.f);
    if (q > bestq) {  // argmax: first maximum
      bestq = q;
      besta = a;
    }
  }
  const float lt = zl ? head_logit(tg, hb_tg, A, Z, besta, lane, mtg) : -INFINITY;
  const float mx = wmax(lt);
  const float e = zl ? expf(lt - mx) : 0.f;
  const float p = e / wsum(e);
  float tz = rew[b] + gamma_n * (1.0f - done[b]) * sup;
  tz = fminf(fmaxf(tz, vmin), vmax);
  const float bb = (tz - vmin) / dz;
  const float lf = floorf(bb), uf = ceilf(bb);
  const int li = (int)lf, ui = (int)uf;
  // m[l] += p (u - b); m[u] += p (b - l): gathered per destination atom, in source order
  float acc = 0.f;
  for (int j = 0; j < Z; ++j) {
    const int lj = __shfl(li, j), uj = __shfl(ui, j);
    const float pj = __shfl(p, j), bj = __shfl(bb, j), lfj = __shfl(lf, j), ufj = __shfl(uf, j);
    if (lj == lane) acc += pj * (ufj - bj);
    if (uj == lane) acc += pj * (bj - lfj);
  }
  if (zl) m[(long long)b * Z + lane] = acc;
  if (lane == 0) a_next[b] = besta;
}

// expected Q per action (drqeps.py:80-84: softmax over atoms . support), one wave per sample
__global__ void q_values_kernel(const float* __restrict__ hc, int ldh, const float* __restrict__ hb, int A, int Z,
                                float vmin, float vmax, float* __restrict__ q, int B) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (b >= B) return;
  const float* h = hc + (long long)b * ldh;
  const bool zl = lane < Z;
  const float sup = vmin + (vmax - vmin) / (float)(Z - 1) * (float)lane;
  float madv = 0.f;
  if (zl) {
#pragma unroll 6
    for (int a = 0; a < A; ++a) madv += h[a * Z + lane] + hb[a * Z + lane];
    madv /= (float)A;
  }
  for (int a = 0; a < A; ++a) {
    const float l = zl ? head_logit(h, hb, A, Z, a, lane, madv) : -INFINITY;
    const float mx = wmax(l);
    const float e = zl ? expf(l - mx) : 0.f;
    const float se = wsum(e);
    const float qa = wsum(zl ? (e / se) * sup : 0.f);
    if (lane == 0) q[(long long)b * A + a] = qa;
  }
}

// Cross entropy at the taken action and its gradient (drqeps.py:300-309): per sample
// loss_b = -sum_z m log_softmax(logit[act]); d logit[act] = (softmax sum(m) - m) / B, then through
// the dueling combination: d val = d logit[act], d adv[a] = d logit[act] (delta(a, act) - 1 / A).
// dh[b][ldh] = [d adv | d val]; per-sample loss and mean logit into small arrays.
__global__ void c51_loss_kernel(const float* __restrict__ hc, int ldh, const float* __restrict__ hb, int A, int Z,
                                const int* __restrict__ act, const float* __restrict__ m, float inv_b,
                                float* __restrict__ dh, float* __restrict__ loss_b, float* __restrict__ logit_b,
                                int B) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (b >= B) return;
  const float* h = hc + (long long)b * ldh;
  const bool zl = lane < Z;
  float madv = 0.f;
  if (zl) {
#pragma unroll 6
    for (int a = 0; a < A; ++a) madv += h[a * Z + lane] + hb[a * Z + lane];
    madv /= (float)A;
  }
  const int ab = act[b];
  const float l = zl ? head_logit(h, hb, A, Z, ab, lane, madv) : -INFINITY;
  const float mx = wmax(l);
  const float e = zl ? expf(l - mx) : 0.f;
  const float se = wsum(e);
  const float lse = mx + logf(se);
  const float mz = zl ? m[(long long)b * Z + lane] : 0.f;
  const float lossb = -wsum(zl ? mz * (l - lse) : 0.f);
  const float msum = wsum(mz);
  const float g = zl ? ((e / se) * msum - mz) * inv_b : 0.f;
  float* d = dh + (long long)b * ldh;
  if (zl) {
    d[A * Z + lane] = g;
    for (int a = 0; a < A; ++a) d[a * Z + lane] = g * ((a == ab ? 1.0f : 0.0f) - 1.0f / (float)A);
  }
  const float ls = wsum(zl ? l : 0.f);
  if (lane == 0) {
    loss_b[b] = lossb;
    logit_b[b] = ls;
  }
}

// embedding backward: dE[t] = sum over the task's rows of d(e / (|e| + 1e-8)) / de (rows in order)
__global__ void embed_bwd_kernel(const float* __restrict__ dfeat, int ldf, int off, const float* __restrict__ emb,
                                 int D, const int* __restrict__ task, int B, float* __restrict__ demb) {
  // the rows of task t listed once in LDS (all task ids loaded together: read one at a time under
  // the row loop's branch, each load was waited for), then the same per-row arithmetic in row order
  __shared__ int rows[1024];
  __shared__ int nrows;
  const int t = blockIdx.x, lane = threadIdx.x;
  float s = 0.f;
  for (int d = lane; d < D; d += 64) s += emb[t * D + d] * emb[t * D + d];
  s = wsum(s);
  const float n = sqrtf(s), ne = n + 1e-8f;
  for (int b0 = 0; b0 < B; b0 += 1024) {
    const int nb = min(1024, B - b0);
    if (lane == 0) nrows = 0;
    __syncthreads();
    // ordered compaction: each lane owns consecutive rows, a prefix over the lanes' counts
    const int per = (nb + 63) / 64, lo = min(lane * per, nb), hi = min(lo + per, nb);
    int cnt = 0;
    for (int b = lo; b < hi; ++b) cnt += task[b0 + b] == t;
    int pre = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(pre, o);
      if (lane >= o) pre += u;
    }
    int w = pre - cnt;
    for (int b = lo; b < hi; ++b)
      if (task[b0 + b] == t) rows[w++] = b0 + b;
    if (lane == 63) nrows = pre;
    __syncthreads();
    const int m = nrows;
    // D <= 64 (drq_create): lane d holds element d; four rows' loads and reductions in flight at once,
    // their contributions added in row order
    const bool on = lane < D;
    const float e = on ? emb[t * D + lane] : 0.f;
    float acc = b0 == 0 || !on ? 0.f : demb[t * D + lane];
    for (int k2 = 0; k2 < m; k2 += 4) {
      float gv[4], wg[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float* g = dfeat + (long long)rows[min(k2 + u, m - 1)] * ldf + off;
        gv[u] = on ? g[lane] : 0.f;
        wg[u] = e * gv[u];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) wg[u] = wsum(wg[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (k2 + u < m) acc += gv[u] / ne - e * wg[u] / (n * ne * ne);
    }
    if (on) demb[t * D + lane] = acc;
    __syncthreads();
  }
}

// d enc = d feat[:, :nenc] * [enc > 0]   (the encoder's final ReLU)
__global__ void enc_grad_kernel(const float* __restrict__ dfeat, int ldf, const float* __restrict__ enc, int nenc,
                                float* __restrict__ denc, int B) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (long long)B * nenc) return;
  const long long b = i / nenc;
  const int k = (int)(i - b * nenc);
  denc[i] = enc[i] > 0.f ? dfeat[b * ldf + k] : 0.f;
}

// ------------------------------------------------------------------ AdamW + Polyak + norms
// optax.adamw (weight decay on every leaf, no clip); target = tau p + (1 - tau) target;
// sumsq partials of g and of the PRE-update p (the logged norms)
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, float* __restrict__ mu,
                                                    float* __restrict__ nu, const float* __restrict__ g,
                                                    float* __restrict__ tgt, long long n, float lr, float b1,
                                                    float b2, float eps, float wd, float tau, int count,
                                                    float* __restrict__ part) {
  const float bc1 = 1.0f - powf(b1, (float)count), bc2 = 1.0f - powf(b2, (float)count);
  float sg = 0.f, sp = 0.f;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const float gi = g[i], pi = p[i];
    sg += gi * gi;
    sp += pi * pi;
    const float m = (1.0f - b1) * gi + b1 * mu[i];
    const float v = (1.0f - b2) * (gi * gi) + b2 * nu[i];
    mu[i] = m;
    nu[i] = v;
    const float u = (m / bc1) / (sqrtf(v / bc2) + eps) + wd * pi;
    const float np = pi + (-lr) * u;
    p[i] = np;
    tgt[i] = tau * np + (1.0f - tau) * tgt[i];
  }
  __shared__ float red[2][4];
  sg = wsum(sg);
  sp = wsum(sp);
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = sg;
    red[1][threadIdx.x >> 6] = sp;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    part[2 * blockIdx.x + 1] = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  }
}

// logs: [mean online logit, |g|, |p_pre|, loss]
__global__ void drq_logs_kernel(const float* __restrict__ part, int G, const float* __restrict__ loss_b,
                                const float* __restrict__ logit_b, int B, int Z, float* __restrict__ logs) {
  __shared__ double red[4][4];
  double a = 0, b = 0, c = 0, d = 0;
  for (int i = threadIdx.x; i < G; i += 256) {
    a += part[2 * i];
    b += part[2 * i + 1];
  }
  for (int i = threadIdx.x; i < B; i += 256) {
    c += loss_b[i];
    d += logit_b[i];
  }
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o);
    b += __shfl_xor(b, o);
    c += __shfl_xor(c, o);
    d += __shfl_xor(d, o);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = a;
    red[1][threadIdx.x >> 6] = b;
    red[2][threadIdx.x >> 6] = c;
    red[3][threadIdx.x >> 6] = d;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double r[4];
    for (int k = 0; k < 4; ++k) r[k] = (red[k][0] + red[k][1]) + (red[k][2] + red[k][3]);
    logs[0] = (float)(r[3] / ((double)B * Z));
    logs[1] = (float)sqrt(r[0]);
    logs[2] = (float)sqrt(r[1]);
    logs[3] = (float)(r[2] / B);
  }
}

// ------------------------------------------------------------------ compute_weights (drqeps.py:353-482)
// Internal layout -> flax ravel order of one gradient (a row of the per-task matrix).  Segment
// table entries: (flax offset, internal offset, count, internal row stride, rows).
__global__ void flax_gather_kernel(const float* __restrict__ g, const long long* __restrict__ map,
                                   float* __restrict__ out) {
  const long long* m = map + 5 * blockIdx.y;
  const long long f = m[0], i0 = m[1], n = m[2], ld = m[3], rows = m[4];
  for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < n * rows; e += (long long)gridDim.x * 256) {
    const long long r = e / n, c = e - r * n;
    out[f + e] = g[i0 + r * (ld ? ld : n) + c];
  }
}

// jax.random.normal(PRNGKey(seed), shape) element at linear index `lin` (jax 0.5.3 defaults:
// threefry2x32 with jax_threefry_partitionable = True, so the element's bits are
// threefry2x32(key = (0, seed), counter = (lin >> 32, lin & 0xffffffff)) as out0 ^ out1; then
// _uniform on [nextafter(-1, 0), 1) and sqrt(2) * erf_inv with XLA's single-precision erf_inv
// (Giles' polynomial, w = -log1p(-x^2)).
__device__ inline unsigned rotl32(unsigned x, int r) { return (x << r) | (x >> (32 - r)); }

__device__ inline unsigned threefry_bits(unsigned k0, unsigned k1, unsigned c0, unsigned c1) {
  const unsigned k2 = k0 ^ k1 ^ 0x1BD11BDAu;
  unsigned x0 = c0 + k0, x1 = c1 + k1;
#define TF_ROUND(r) \
  x0 += x1;         \
  x1 = rotl32(x1, r); \
  x1 ^= x0;
#define TF_A TF_ROUND(13) TF_ROUND(15) TF_ROUND(26) TF_ROUND(6)
#define TF_B TF_ROUND(17) TF_ROUND(29) TF_ROUND(16) TF_ROUND(24)
  TF_A x0 += k1; x1 += k2 + 1u;
  TF_B x0 += k2; x1 += k0 + 2u;
  TF_A x0 += k0; x1 += k1 + 3u;
  TF_B x0 += k1; x1 += k2 + 4u;
  TF_A x0 += k2; x1 += k0 + 5u;
#undef TF_A
#undef TF_B
#undef TF_ROUND
  return x0 ^ x1;
}

__device__ inline float jax_normal(unsigned seed, unsigned long long lin) {
  const unsigned bits = threefry_bits(0u, seed, (unsigned)(lin >> 32), (unsigned)lin);
  const float f = __uint_as_float((bits >> 9) | 0x3f800000u) - 1.0f;
  const float lo = -0.99999994f;  // nextafter(-1, 0)
  const float x = fmaxf(lo, f * 2.0f + lo);  // (maxval - minval) rounds to 2 in float32
  float w = -log1pf(-x * x);
  const bool lt = w < 5.0f;
  w = lt ? w - 2.5f : sqrtf(w) - 3.0f;
  float p = lt ? 2.81022636e-08f : -0.000200214257f;
  p = (lt ? 3.43273939e-07f : 0.000100950558f) + p * w;
  p = (lt ? -3.5233877e-06f : 0.00134934322f) + p * w;
  p = (lt ? -4.39150654e-06f : -0.00367342844f) + p * w;
  p = (lt ? 0.00021858087f : 0.00573950773f) + p * w;
  p = (lt ? -0.00125372503f : -0.0076224613f) + p * w;
  p = (lt ? -0.00417768164f : 0.00943887047f) + p * w;
  p = (lt ? 0.246640727f : 1.00167406f) + p * w;
  p = (lt ? 1.50140941f : 2.83297682f) + p * w;
  return 1.41421354f * (p * x);
}

// project_grad (drqeps.py:428-448) for up to JL_T task rows at once, each random matrix element
// generated once and used for every task: part[ks][t][j] = sum_{k in split ks} G[t][k] N(k, j) with
// N(k, j) = normal(PRNGKey(seed + k / chunk))[(k % chunk) * D + j].  One lane per output column j;
// the G tile [JL_K][JL_T] in LDS (broadcast reads).
constexpr int JL_T = 32, JL_K = 64;

__global__ __launch_bounds__(256) void jl_project_kernel(const float* __restrict__ G, long long ldg, int T,
                                                         long long P, int D, long long chunk, int seed,
                                                         long long kper, float* __restrict__ part) {
  __shared__ float gs[JL_K][JL_T];
  const int j = blockIdx.x * 256 + threadIdx.x;
  const long long k0 = (long long)blockIdx.y * kper, k1 = k0 + kper < P ? k0 + kper : P;
  float acc[JL_T];
#pragma unroll
  for (int t = 0; t < JL_T; ++t) acc[t] = 0.f;
  for (long long kb = k0; kb < k1; kb += JL_K) {
    __syncthreads();
    for (int e = threadIdx.x; e < JL_K * JL_T; e += 256) {
      const int kk = e / JL_T, t = e - kk * JL_T;
      const long long k = kb + kk;
      gs[kk][t] = (t < T && k < k1) ? G[(long long)t * ldg + k] : 0.f;
    }
    __syncthreads();
    if (j < D) {
      const int kn = (int)(k1 - kb < JL_K ? k1 - kb : JL_K);
      for (int kk = 0; kk < kn; ++kk) {
        const long long k = kb + kk;
        const long long c = k / chunk;
        const float n = jax_normal((unsigned)(seed + c), (unsigned long long)(k - c * chunk) * D + j);
        const float4* row = reinterpret_cast<const float4*>(&gs[kk][0]);
#pragma unroll
        for (int q = 0; q < JL_T / 4; ++q) {
          const float4 g4 = row[q];
          acc[4 * q] += g4.x * n;
          acc[4 * q + 1] += g4.y * n;
          acc[4 * q + 2] += g4.z * n;
          acc[4 * q + 3] += g4.w * n;
        }
      }
    }
  }
  if (j < D)
    for (int t = 0; t < T && t < JL_T; ++t) part[((long long)blockIdx.y * JL_T + t) * D + j] = acc[t];
}

// out[t][j] = (sum over splits, in order, in double) / sqrt(D)
__global__ void jl_reduce_kernel(const float* __restrict__ part, int splits, int T, int D, float div,
                                 float* __restrict__ out, long long ldo) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= (long long)T * D) return;
  const int t = (int)(e / D), j = (int)(e - (long long)t * D);
  double s = 0.0;
  for (int k = 0; k < splits; ++k) s += part[((long long)k * JL_T + t) * D + j];
  out[(long long)t * ldo + j] = (float)(s / div);
}

}  // namespace

// ------------------------------------------------------------------ launchers
static unsigned blocks(long long n, int t = 256) { return (unsigned)((n + t - 1) / t); }

void atari_sample(const unsigned char* store, const unsigned char* nstore, const int* act, const float* rew,
                  const float* done, const float* trunc, const double* minmax, const int* idx, long long cap, int T,
                  int n, int img_bytes, int nstep, int full, int pos, int guard, double eps, unsigned char* obs,
                  unsigned char* nobs, int* act_out, float* rew_out, float* done_out, float* trunc_out, int* task_out,
                  hipStream_t st) {
  AtariSampleParams p{store, nstore, act, rew, done, trunc, minmax, idx, cap, T, n, img_bytes / 16, nstep, full, pos,
                      guard, eps, obs, nobs, act_out, task_out, rew_out, done_out, trunc_out, nullptr, nullptr};
  hipLaunchKernelGGL(atari_sample_kernel, dim3(4, n * T), dim3(256), 0, st, p);
}

void atari_sample_rows(const unsigned char* store, const unsigned char* nstore, const int* act, const float* rew,
                       const float* done, const float* trunc, const double* minmax, const long long* slots,
                       const int* tasks, int rows, long long cap, int T, int img_bytes, int nstep, double eps, unsigned char* obs,
                       unsigned char* nobs, int* act_out, float* rew_out, float* done_out, float* trunc_out,
                       int* task_out, hipStream_t st) {
  AtariSampleParams p{store, nstore, act, rew, done, trunc, minmax, nullptr, cap, T, 1, img_bytes / 16, nstep, 0, 0,
                      0, eps, obs, nobs, act_out, task_out, rew_out, done_out, trunc_out, slots, tasks};
  hipLaunchKernelGGL(atari_sample_kernel, dim3(4, rows), dim3(256), 0, st, p);
}

void aug_draw(unsigned long long seed, unsigned long long ctr, int B, int pad, int* crop_o, float* noise_o,
              int* crop_n, float* noise_n, hipStream_t st) {
  hipLaunchKernelGGL(aug_draw_kernel, dim3(blocks(2LL * B)), dim3(256), 0, st, seed, ctr, B, 2 * pad, crop_o, noise_o,
                     crop_n, noise_n);
}

void augment(const unsigned char* obs, const int* crop, const float* noise, float* out, int B, int C, int H, int W,
             int pad, hipStream_t st) {
  const long long n = (long long)B * C * H * W;
  hipLaunchKernelGGL(augment_kernel, dim3(blocks(n)), dim3(256), 0, st, obs, crop, noise, out, B, C, H, W, pad);
}

void augment3(const unsigned char* obs, const int* crop_o, const float* noise_o, const unsigned char* nobs,
              const int* crop_n, const float* noise_n, float* out, int B, int C, int H, int W, int pad, hipStream_t st) {
  const long long n = 2LL * B * H * W;  // one lane per output pixel of the obs and next-obs halves
  hipLaunchKernelGGL(augment3_kernel, dim3(blocks(n)), dim3(256), 0, st, obs, crop_o, noise_o, nobs, crop_n, noise_n,
                     out, B, C, H, W, pad);
}

#define CONV_CASES(M)                   \
  M(4, 8) M(8, 8) M(8, 16) M(16, 16)

bool conv_supported(int ci, int co) {
#define C_OK(a, b) if (ci == a && co == b) return true;
  CONV_CASES(C_OK)
#undef C_OK
  return false;
}

// channels per lane (measured, rocprofv3 per-kernel sums): the forward keeps every output channel
// of a pixel in one lane (splitting re-reads the input patch per group) while the launch has enough
// waves to hide its latency; the data gradient splits 16 input channels into groups of 4 (4x the
// waves for the same dout reads, 1.4x faster there).  g_drq_fwd_g / g_drq_bwd_g > 0 force a group
// (experiments, mtsac_debug_drq_groups).
int g_drq_fwd_g = 0, g_drq_bwd_g = 0;
static int conv_fwd_group(int co, long long npix) {
  if (g_drq_fwd_g > 0 && co % g_drq_fwd_g == 0) return g_drq_fwd_g;
  return co;
}
static int conv_bwd_group(int ci) {
  if (g_drq_bwd_g > 0 && ci % g_drq_bwd_g == 0) return g_drq_bwd_g;
  return ci == 16 ? 4 : ci;
}

// f32-MFMA convolutions (bit 1 forward, 2 data grad, 4 weight grad); the VALU kernels otherwise
// Measured, not kept (profiles/r4c_*, r4d_*: batch 256, 303-395 vs 494 DrQ steps/s): the f32 MFMA has
// the packed-FMA rate, so it can only win on operand delivery, and these kernels -- operands one fp32
// per lane straight from L1/L2, 16-column tiles half empty at 8 channels -- lose to the VALU kernels'
// scalar-operand FMAs (weight grads 2-3x slower, forwards 1.2-2x).  Opt-in experiments only.
int g_drq_mfma = [] {
  const char* e = getenv("MTSAC_DRQ_MFMA");
  return e ? (atoi(e) & 7) : 0;
}();
constexpr int MFMA_TW = 4;  // 16-pixel tiles per wave of conv_mfma_kernel

// Row-tile forward / data-gradient geometry (conv_rows_kernel): for NG = 1, 2, 4 output-channel groups
// (CG = KO / NG >= 4 channels a lane) a tile holds up to 256 / NG pixels; R = the rows that fit,
// balanced over the image; the NG with the best-filled tiles wins (ties: fewer groups, less
// re-reading).  NG = 0: no fit (W < 2, or a row too wide), the pixel kernels run instead.
static ConvGeo conv_geo(int H, int W, int KI, int KO, int* ng_out) {
  ConvGeo best{H, W, 0, (W + 2) * KI, 0, 0u, 0u};
  double best_u = 0.0;
  *ng_out = 0;
  if (W < 2) return best;
  for (int ng = 1; ng <= 4; ng *= 2) {
    if (KO % ng || KO / ng < 4) continue;
    const int cap = 256 / ng;
    int R = std::min({H, cap / W, CR_LDS / best.SR - 2});
    if (R < 1) continue;
    const int n = (H + R - 1) / R;
    R = (H + n - 1) / n;
    const double u = (double)(R * W) / cap;
    if (u > best_u + 1e-9) {
      best_u = u;
      best.R = R;
      best.n = n;
      *ng_out = ng;
    }
  }
  best.magic = (unsigned)((0x100000000ULL + (unsigned)W - 1) / (unsigned)W);
  best.magic2 = (unsigned)((0x100000000ULL + (unsigned)W + 1) / (unsigned)(W + 2));
  return best;
}
// a forced channel group (mtsac_debug_drq_groups), the MFMA experiment or the legacy mask selects the
// one-lane-per-pixel kernels
static bool conv_rows_on(int ng, int forced_group, int bit) {
  return ng > 0 && forced_group == 0 && !(g_drq_mfma & bit) && !(g_drq_legacy & bit);
}

// split2h MFMA geometry (conv_h2_kernel): the tallest balanced row tile whose two fp16 planes fit
// CH_LDS (the staging slots then fit too); R = 0 (the VALU kernels) for W < 2 or too wide a row
static ConvGeo conv_h2_geo(int H, int W, int KI) {
  ConvGeo g{H, W, 0, 0, 0, 0u, 0u};
  if (W < 2) return g;
  const int R = std::min(H, CH_LDS / ((W + 2) * KI) - 2);
  if (R < 1) return g;
  g.n = (H + R - 1) / R;
  g.R = (H + g.n - 1) / g.n;
  g.magic = (unsigned)((0x100000000ULL + (unsigned)W - 1) / (unsigned)W);
  g.magic2 = (unsigned)((0x100000000ULL + (unsigned)W + 1) / (unsigned)(W + 2));
  return g;
}
// the split2h MFMA convs (legacy bit 16: the VALU kernels).  Measured per shape (batch 256,
// profiles/r6w_drq_h2/conv_bench.txt, us per launch, split2h vs the VALU choice): they win with 16
// input channels on the small images (forward 21 x 21: 27.3 vs 30.7, 11 x 11: 9.5 vs 9.9; data grad
// 11.9 vs 14.0, 7.2 vs 8.0) and lose elsewhere (42 x 42 8 -> 8 forward 46.5 vs 30.1; the data grads
// at 42 and 84: 22-58 vs 14-32): the per-block weight gather and split and the staging's max
// reduction cost more than the MFMAs save there.  They run for KI = 16, W <= 32.
static bool conv_h2_on(const ConvGeo& g, int KI, int bit) {
  const bool shape = (KI == 16 && g.W <= 32) || (g_drq_legacy & 32);  // bit 32: every supported shape
  return g.R > 0 && shape && !(g_drq_legacy & 16) && !(g_drq_legacy & bit) && !(g_drq_mfma & bit);
}

void conv_fwd(const float* in, const float* w, const float* bias, const float* res, float* out, int B, int H, int W,
              int ci, int co, bool relu_in, hipStream_t st, const float* w2, const float* bias2, int B1) {
  const long long npix = (long long)B * H * W;
  const int G = conv_fwd_group(co, npix);
  if (w2 == nullptr || B1 < 0 || B1 > B) {  // one parameter set
    w2 = w;
    bias2 = bias;
    B1 = B;
  }
  if (ci >= 8 && g_drq_fwd_g == 0) {
    const ConvGeo geo = conv_h2_geo(H, W, ci);
    if (conv_h2_on(geo, ci, 1)) {
      const dim3 gr((unsigned)(B * geo.n)), tb(256);
#define C_FH(a, b)                                                                                                   \
  if (ci == a && co == b) {                                                                                          \
    if (relu_in && res) hipLaunchKernelGGL((conv_h2_kernel<a, b, true, true, false, true>), gr, tb, 0, st, in, w, bias, w2, bias2, B1, nullptr, res, out, geo); \
    else if (relu_in) hipLaunchKernelGGL((conv_h2_kernel<a, b, true, true, false, false>), gr, tb, 0, st, in, w, bias, w2, bias2, B1, nullptr, res, out, geo); \
    else if (res) hipLaunchKernelGGL((conv_h2_kernel<a, b, true, false, false, true>), gr, tb, 0, st, in, w, bias, w2, bias2, B1, nullptr, res, out, geo); \
    else hipLaunchKernelGGL((conv_h2_kernel<a, b, true, false, false, false>), gr, tb, 0, st, in, w, bias, w2, bias2, B1, nullptr, res, out, geo); \
    return;                                                                                                          \
  }
      C_FH(8, 8) C_FH(8, 16) C_FH(16, 16)
#undef C_FH
    }
  }
  {
    int ng = 0;
    const ConvGeo geo = conv_geo(H, W, ci, co, &ng);
    if (conv_rows_on(ng, g_drq_fwd_g, 1)) {
      const dim3 gr((unsigned)(B * geo.n)), tb(256);
#define C_FR_G(a, b, cg)                                                                                            \
  if (relu_in && res) hipLaunchKernelGGL((conv_rows_kernel<a, b, cg, true, true, false, true>), gr, tb, 0, st, in, w, bias, w2, bias2, B1, nullptr, res, out, geo); \
  else if (relu_in) hipLaunchKernelGGL((conv_rows_kernel<a, b, cg, true, true, false, false>), gr, tb, 0, st, in, w, bias, w2, bias2, B1, nullptr, res, out, geo); \
  else if (res) hipLaunchKernelGGL((conv_rows_kernel<a, b, cg, true, false, false, true>), gr, tb, 0, st, in, w, bias, w2, bias2, B1, nullptr, res, out, geo); \
  else hipLaunchKernelGGL((conv_rows_kernel<a, b, cg, true, false, false, false>), gr, tb, 0, st, in, w, bias, w2, bias2, B1, nullptr, res, out, geo);
#define C_FR(a, b)                                   \
  if (ci == a && co == b) {                          \
    if (ng == 1) { C_FR_G(a, b, b) }                 \
    else if (ng == 2) { C_FR_G(a, b, b / 2) }        \
    else if constexpr (b >= 16) { C_FR_G(a, b, b / 4) } \
    return;                                          \
  }
      CONV_CASES(C_FR)
#undef C_FR
#undef C_FR_G
    }
  }
  if (g_drq_mfma & 1) {
    constexpr int PB = 64 * MFMA_TW;
    const long long n1 = (long long)B1 * H * W;
    const dim3 gm((unsigned)((n1 + PB - 1) / PB + (npix - n1 + PB - 1) / PB)), tm(256);
#define C_FWDM(a, b)                                                                                                 \
  if (ci == a && co == b) {                                                                                          \
    if (relu_in && res) hipLaunchKernelGGL((conv_mfma_kernel<a, b, true, true, true, MFMA_TW>), gm, tm, 0, st, in, w, bias, w2, bias2, nullptr, res, out, B, B1, H, W); \
    else if (relu_in) hipLaunchKernelGGL((conv_mfma_kernel<a, b, true, true, false, MFMA_TW>), gm, tm, 0, st, in, w, bias, w2, bias2, nullptr, res, out, B, B1, H, W); \
    else if (res) hipLaunchKernelGGL((conv_mfma_kernel<a, b, true, false, true, MFMA_TW>), gm, tm, 0, st, in, w, bias, w2, bias2, nullptr, res, out, B, B1, H, W); \
    else hipLaunchKernelGGL((conv_mfma_kernel<a, b, true, false, false, MFMA_TW>), gm, tm, 0, st, in, w, bias, w2, bias2, nullptr, res, out, B, B1, H, W); \
    return;                                                                                                          \
  }
    CONV_CASES(C_FWDM)
#undef C_FWDM
  }
  const long long n1 = (long long)B1 * H * W;
  const dim3 g(blocks(n1) + blocks(npix - n1), co / G), t(256);
#define C_FWD_G(a, b, cg)                                                                                           \
  if (relu_in && res) hipLaunchKernelGGL((conv_fwd_kernel<a, b, cg, true, true>), g, t, 0, st, in, w, bias, w2, bias2, res, out, B, B1, H, W); \
  else if (relu_in) hipLaunchKernelGGL((conv_fwd_kernel<a, b, cg, true, false>), g, t, 0, st, in, w, bias, w2, bias2, res, out, B, B1, H, W); \
  else if (res) hipLaunchKernelGGL((conv_fwd_kernel<a, b, cg, false, true>), g, t, 0, st, in, w, bias, w2, bias2, res, out, B, B1, H, W); \
  else hipLaunchKernelGGL((conv_fwd_kernel<a, b, cg, false, false>), g, t, 0, st, in, w, bias, w2, bias2, res, out, B, B1, H, W);
#define C_FWD(a, b)                   \
  if (ci == a && co == b) {           \
    if (G == b) { C_FWD_G(a, b, b) }  \
    else if (G == 8) { C_FWD_G(a, b, 8) } \
    else { C_FWD_G(a, b, 4) }         \
    return;                           \
  }
  CONV_CASES(C_FWD)
#undef C_FWD
#undef C_FWD_G
}

void conv_bwd_data(const float* dout, const float* w, const float* mask, const float* dres, float* din, int B, int H,
                   int W, int ci, int co, hipStream_t st) {
  const long long npix = (long long)B * H * W;
  if (co >= 8 && g_drq_bwd_g == 0) {  // the transposed conv on split2h MFMA: KI = co, KO = ci
    const ConvGeo geo = conv_h2_geo(H, W, co);
    if (conv_h2_on(geo, co, 2)) {
      const dim3 gr((unsigned)(B * geo.n)), tb(256);
#define C_BH(a, b)                                                                                                   \
  if (ci == a && co == b) {                                                                                          \
    if (mask && dres) hipLaunchKernelGGL((conv_h2_kernel<b, a, false, false, true, true>), gr, tb, 0, st, dout, w, nullptr, w, nullptr, B, mask, dres, din, geo); \
    else if (mask) hipLaunchKernelGGL((conv_h2_kernel<b, a, false, false, true, false>), gr, tb, 0, st, dout, w, nullptr, w, nullptr, B, mask, dres, din, geo); \
    else if (dres) hipLaunchKernelGGL((conv_h2_kernel<b, a, false, false, false, true>), gr, tb, 0, st, dout, w, nullptr, w, nullptr, B, mask, dres, din, geo); \
    else hipLaunchKernelGGL((conv_h2_kernel<b, a, false, false, false, false>), gr, tb, 0, st, dout, w, nullptr, w, nullptr, B, mask, dres, din, geo); \
    return;                                                                                                          \
  }
      C_BH(4, 8) C_BH(8, 8) C_BH(8, 16) C_BH(16, 16)
#undef C_BH
    }
  }
  {  // the transposed conv: KI = co (dout channels), KO = ci
    int ng = 0;
    const ConvGeo geo = conv_geo(H, W, co, ci, &ng);
    // measured (profiles/r6o_drq/conv_bench.txt): the row-tile data grad wins with 16 dout channels
    // from 21 x 21 up (21 x 21: 13.6 vs 28.2 us, 42 x 42 8 -> 16: 25.0 vs 27.9) and loses with 8 (42 x 42:
    // 15.2 vs 13.9) and at 11 x 11 (8.5 vs 7.9): it runs for co = 16, W >= 16
    if (((co >= 16 && W >= 16) || (g_drq_legacy & 8)) && conv_rows_on(ng, g_drq_bwd_g, 2)) {
      const dim3 gr((unsigned)(B * geo.n)), tb(256);
#define C_BR_G(a, b, cg)                                                                                            \
  if (mask && dres) hipLaunchKernelGGL((conv_rows_kernel<b, a, cg, false, false, true, true>), gr, tb, 0, st, dout, w, nullptr, w, nullptr, B, mask, dres, din, geo); \
  else if (mask) hipLaunchKernelGGL((conv_rows_kernel<b, a, cg, false, false, true, false>), gr, tb, 0, st, dout, w, nullptr, w, nullptr, B, mask, dres, din, geo); \
  else if (dres) hipLaunchKernelGGL((conv_rows_kernel<b, a, cg, false, false, false, true>), gr, tb, 0, st, dout, w, nullptr, w, nullptr, B, mask, dres, din, geo); \
  else hipLaunchKernelGGL((conv_rows_kernel<b, a, cg, false, false, false, false>), gr, tb, 0, st, dout, w, nullptr, w, nullptr, B, mask, dres, din, geo);
#define C_BR(a, b)                                   \
  if (ci == a && co == b) {                          \
    if (ng == 1) { C_BR_G(a, b, a) }                 \
    else if constexpr (a >= 8) {                     \
      if (ng == 2) { C_BR_G(a, b, a / 2) }           \
      else if constexpr (a >= 16) { C_BR_G(a, b, a / 4) } \
    }                                                \
    return;                                          \
  }
      CONV_CASES(C_BR)
#undef C_BR
#undef C_BR_G
    }
  }
  if (g_drq_mfma & 2) {  // K channels = co, N = ci
    constexpr int PB = 64 * MFMA_TW;
    const dim3 gm((unsigned)((npix + PB - 1) / PB)), tm(256);
#define C_BDM(a, b)                                                                                                  \
  if (ci == a && co == b) {                                                                                          \
    if (dres) hipLaunchKernelGGL((conv_mfma_kernel<b, a, false, false, true, MFMA_TW>), gm, tm, 0, st, dout, w, nullptr, w, nullptr, mask, dres, din, B, B, H, W); \
    else hipLaunchKernelGGL((conv_mfma_kernel<b, a, false, false, false, MFMA_TW>), gm, tm, 0, st, dout, w, nullptr, w, nullptr, mask, dres, din, B, B, H, W); \
    return;                                                                                                          \
  }
    CONV_CASES(C_BDM)
#undef C_BDM
  }
  const int G = conv_bwd_group(ci);
  const dim3 g(blocks(npix), ci / G), t(256);
#define C_BD_G(a, b, cg)                                                                                            \
  if (mask && dres) hipLaunchKernelGGL((conv_bwd_data_kernel<a, b, cg, true, true>), g, t, 0, st, dout, w, mask, dres, din, B, H, W); \
  else if (mask) hipLaunchKernelGGL((conv_bwd_data_kernel<a, b, cg, true, false>), g, t, 0, st, dout, w, mask, dres, din, B, H, W); \
  else if (dres) hipLaunchKernelGGL((conv_bwd_data_kernel<a, b, cg, false, true>), g, t, 0, st, dout, w, mask, dres, din, B, H, W); \
  else hipLaunchKernelGGL((conv_bwd_data_kernel<a, b, cg, false, false>), g, t, 0, st, dout, w, mask, dres, din, B, H, W);
#define C_BD(a, b)                   \
  if (ci == a && co == b) {          \
    if (G == a) { C_BD_G(a, b, a) }  \
    else if (G == 8) { if constexpr (a >= 8) { C_BD_G(a, b, 8) } } \
    else { C_BD_G(a, b, 4) }         \
    return;                          \
  }
  CONV_CASES(C_BD)
#undef C_BD
#undef C_BD_G
}

// Row-tile weight gradients (conv_wgrad_rows_kernel): the tallest tile whose staging fits the
// per-thread slots and the kernel's LDS, shortened until the batch gives >= 512 tiles (two blocks
// per CU), then balanced (equal row counts per image); R = 0 when even one row does not fit (very wide
// images) or W < 2 (the magic division), where the im2col kernel runs instead.
static int wg_lds_floats(int ci, int co) {
#define C_WL(a, b) if (ci == a && co == b) return 4 * WgRows<a, b>::LDS4;
  CONV_CASES(C_WL)
#undef C_WL
  return 0;
}
int g_drq_wg_blocks = 0;  // > 0: the row-tile weight grad's grid cap (mtsac_debug_drq_wgrad_blocks)
static WgGeo wgrad_geo(int B, int H, int W, int ci, int co) {
  WgGeo g{H, W, 0, (W + 2) * ci + 4, 0, 0u};
  const int slots = 8 * 256, ldsf = wg_lds_floats(ci, co);
  auto fits = [&](int R) {
    return (R + 2) * (W + 2) * (ci / 4) + R * W * (co / 4) <= slots && (R + 2) * g.SR + R * W * co <= ldsf;
  };
  if (W < 2 || !fits(1)) return g;
  int R = H;
  while (R > 1 && (!fits(R) || (long long)B * ((H + R - 1) / R) < 2 * 256)) --R;
  const int n = (H + R - 1) / R;
  g.R = (H + n - 1) / n;
  g.tiles = B * n;
  g.magic = (unsigned)((0x100000000ULL + (unsigned)W - 1) / (unsigned)W);
  return g;
}
int g_drq_legacy = [] {  // MTSAC_DRQ_LEGACY=mask in the environment: the same selection (A/B runs)
  const char* e = getenv("MTSAC_DRQ_LEGACY");
  return e ? (atoi(e) & 63) : 0;
}();
// Measured per shape (profiles/r6l_drq/conv_bench.txt, batch 256): the row-tile weight grad wins from
// 21 x 21 up (84 x 84 4 -> 8: 41.5 vs 90.1 us) and loses at 11 x 11 (15.5 vs 9.7: one tile per block,
// where the pixel-group tree is most of the work), so it runs for W >= 16
static bool wgrad_rows(const WgGeo& g) {
  return g.R > 0 && (g.W >= 16 || (g_drq_legacy & 8)) && !(g_drq_mfma & 4) && !(g_drq_legacy & 4);
}
static int wgrad_cap(const WgGeo& g) {  // grid cap: 1024 at 84 x 84 (35.6 vs 41.5 us at 512), else 512
  return g_drq_wg_blocks > 0 ? g_drq_wg_blocks : (g.W >= 64 ? 1024 : 512);
}

// im2col kernel: enough 64-pixel tiles in flight per CU to cover the staging loads' latency (the
// partials' reduction is cheap next to them); the MFMA experiment takes chunks of npix / G pixels
int conv_wgrad_blocks(int B, int H, int W, int ci, int co) {
  const WgGeo g = wgrad_geo(B, H, W, ci, co);
  if (wgrad_rows(g)) return std::min(g.tiles, wgrad_cap(g));
  const long long npix = (long long)B * H * W;
  return (int)std::min<long long>(2048, std::max<long long>(1, (npix + 63) / 64));
}

void conv_wgrad(const float* in, const float* dout, float* part, float* dw, float* db, int B, int H, int W, int ci,
                int co, bool relu_in, hipStream_t st, bool defer_sum) {
  const long long npix = (long long)B * H * W;
  const WgGeo geo = wgrad_geo(B, H, W, ci, co);
  const bool rows = wgrad_rows(geo);
  const int G = conv_wgrad_blocks(B, H, W, ci, co);
  const int chunk = (int)(((npix + G - 1) / G + 15) / 16 * 16);
#define C_WG(a, b)                                                                                             \
  if (ci == a && co == b) {                                                                                    \
    if (rows) {                                                                                                \
      if (relu_in) hipLaunchKernelGGL((conv_wgrad_rows_kernel<a, b, true>), dim3(G), dim3(256), 0, st, in, dout, part, geo); \
      else hipLaunchKernelGGL((conv_wgrad_rows_kernel<a, b, false>), dim3(G), dim3(256), 0, st, in, dout, part, geo);      \
    } else if (g_drq_mfma & 4) {                                                                               \
      if (relu_in) hipLaunchKernelGGL((conv_wgrad_mfma_kernel<a, b, true>), dim3(G), dim3(256), 0, st, in, dout, part, B, H, W, chunk); \
      else hipLaunchKernelGGL((conv_wgrad_mfma_kernel<a, b, false>), dim3(G), dim3(256), 0, st, in, dout, part, B, H, W, chunk);      \
    } else if (relu_in) hipLaunchKernelGGL((conv_wgrad_kernel<a, b, true>), dim3(G), dim3(256), 0, st, in, dout, part, B, H, W); \
    else hipLaunchKernelGGL((conv_wgrad_kernel<a, b, false>), dim3(G), dim3(256), 0, st, in, dout, part, B, H, W);        \
  }
  CONV_CASES(C_WG)
#undef C_WG
  if (defer_sum) return;  // summed with the other convs' partials by sum_parts_multi
  const int nw = 9 * ci * co, n = nw + co;
  hipLaunchKernelGGL(sum_parts_kernel, dim3((n + 15) / 16), dim3(256), 0, st, part, G, n, dw, db, nw);
}

int sum_parts_blocks(int ci, int co) { return (9 * ci * co + co + 15) / 16; }

// Microbenchmark (debug entry mtsac_debug_drq_conv_bench): kind 0 forward (ReLU in, residual), 1 data
// gradient (mask, residual), 2 weight-gradient partials; operands uniform in [-1, 1]; returns the mean
// microseconds per launch over iters launches, or < 0 on an allocation failure
double conv_bench(int kind, int B, int H, int W, int ci, int co, int iters) {
  const long long np = (long long)B * H * W;
  const long long nx = np * (kind == 1 ? co : ci), ny = np * (kind == 1 ? ci : co);
  const int G = conv_wgrad_blocks(B, H, W, ci, co);
  const long long nz = kind == 2 ? (long long)G * (9 * ci * co + co) : ny;
  std::vector<float> hx((size_t)std::max({nx, ny, 9LL * ci * co + co}));
  unsigned long long z = 88172645463325252ULL;
  for (float& v : hx) {
    z ^= z << 13; z ^= z >> 7; z ^= z << 17;
    v = (float)((double)(z >> 11) / 9007199254740992.0 * 2.0 - 1.0);
  }
  float *x = nullptr, *y = nullptr, *o = nullptr, *w = nullptr;
  if (hipMalloc(&x, nx * 4) != hipSuccess || hipMalloc(&y, ny * 4) != hipSuccess ||
      hipMalloc(&o, nz * 4) != hipSuccess || hipMalloc(&w, (9LL * ci * co + co) * 4) != hipSuccess)
    return -1.0;
  (void)hipMemcpy(x, hx.data(), nx * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(y, hx.data(), ny * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(w, hx.data(), (9LL * ci * co + co) * 4, hipMemcpyHostToDevice);
  auto run = [&] {
    if (kind == 0) conv_fwd(x, w, w + 9 * ci * co, y, o, B, H, W, ci, co, true, nullptr);
    else if (kind == 1) conv_bwd_data(x, w, y, y, o, B, H, W, ci, co, nullptr);
    else conv_wgrad(x, y, o, nullptr, nullptr, B, H, W, ci, co, true, nullptr, true);
  };
  run();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, nullptr);
  for (int i = 0; i < iters; ++i) run();
  (void)hipEventRecord(e1, nullptr);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(x);
  (void)hipFree(y);
  (void)hipFree(o);
  (void)hipFree(w);
  return 1e3 * ms / iters;
}

void sum_parts_multi(const SumSeg* segs, int nseg, int blocks, hipStream_t st) {
  hipLaunchKernelGGL(sum_parts_multi_kernel, dim3(blocks), dim3(256), 0, st, segs, nseg);
}

void maxpool_fwd(const float* in, float* out, unsigned char* arg, int B, int H, int W, int C, hipStream_t st) {
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const int lo = std::max((Ho - 1) * 2 + 3 - H, 0) / 2;
  const long long n = (long long)B * Ho * Wo * (C / 4);  // C % 4 == 0, B H W C < 2^31 (drq_create)
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(blocks(n)), dim3(256), 0, st, in, out, arg, B, H, W, C, Ho, Wo, lo);
}

void maxpool_bwd(const float* dout, const unsigned char* arg, float* din, int B, int H, int W, int C, hipStream_t st) {
  const int Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  const int lo = std::max((Ho - 1) * 2 + 3 - H, 0) / 2;
  const long long n = (long long)B * H * W * (C / 4);
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(blocks(n)), dim3(256), 0, st, dout, arg, din, B, H, W, C, Ho, Wo, lo);
}

void concat_feat(const float* enc, int nenc, const float* emb, int D, const int* task, int r0, int tmod, float* feat,
                 int ldf, int B, hipStream_t st) {
  hipLaunchKernelGGL(concat_kernel, dim3(B), dim3(256), 0, st, enc, nenc, emb, D, task, r0, tmod, feat, ldf, B);
}

void ln_fwd(const float* x, const float* xb, int ldx, int F, const float* scale, const float* bias, float eps,
            float* y, int ldy, float* xhat, float* rstd, int B, bool relu, hipStream_t st) {
  if (relu)
    hipLaunchKernelGGL(ln_fwd_kernel<true>, dim3((B + 3) / 4), dim3(256), 0, st, x, xb, ldx, F, scale, bias, eps, y, ldy,
                       xhat, rstd, B);
  else
    hipLaunchKernelGGL(ln_fwd_kernel<false>, dim3((B + 3) / 4), dim3(256), 0, st, x, xb, ldx, F, scale, bias, eps, y,
                       ldy, xhat, rstd, B);
}

void ln_bwd(const float* dy, int lddy, const float* y, int ldy, const float* xhat, const float* rstd,
            const float* scale, int F, float* dx, int lddx, float* dscale, float* dbias, int B, bool relu,
            hipStream_t st) {
  if (relu) {
    hipLaunchKernelGGL(ln_bwd_kernel<true>, dim3((B + 3) / 4), dim3(256), 0, st, dy, lddy, y, ldy, xhat, rstd, scale, F,
                       dx, lddx, B);
    hipLaunchKernelGGL(ln_param_grad_kernel<true>, dim3((F + 15) / 16), dim3(256), 0, st, dy, lddy, y, ldy, xhat, F,
                       B, dscale, dbias);
  } else {
    hipLaunchKernelGGL(ln_bwd_kernel<false>, dim3((B + 3) / 4), dim3(256), 0, st, dy, lddy, y, ldy, xhat, rstd, scale,
                       F, dx, lddx, B);
    hipLaunchKernelGGL(ln_param_grad_kernel<false>, dim3((F + 15) / 16), dim3(256), 0, st, dy, lddy, y, ldy, xhat, F,
                       B, dscale, dbias);
  }
}

void colsum_rows(const float* x, int ld, int F, int B, float* out, hipStream_t st) {
  hipLaunchKernelGGL(colsum_rows_kernel, dim3((F + 15) / 16), dim3(256), 0, st, x, ld, F, B, out);
}

void c51_target(const float* hc_on, const float* hc_tg, int ldh, const float* hb_on, const float* hb_tg, int A, int Z,
                const float* rew, const float* done, float gamma_n, float vmin, float vmax, float* m, int* a_next,
                int B, hipStream_t st) {
  hipLaunchKernelGGL(c51_target_kernel, dim3((B + 3) / 4), dim3(256), 0, st, hc_on, hc_tg, ldh, hb_on, hb_tg, A, Z, rew,
                     done, gamma_n, vmin, vmax, m, a_next, B);
}

void q_values(const float* hc, int ldh, const float* hb, int A, int Z, float vmin, float vmax, float* q, int B,
              hipStream_t st) {
  hipLaunchKernelGGL(q_values_kernel, dim3((B + 3) / 4), dim3(256), 0, st, hc, ldh, hb, A, Z, vmin, vmax, q, B);
}

void c51_loss(const float* hc, int ldh, const float* hb, int A, int Z, const int* act, const float* m, float* dh,
              float* loss_b, float* logit_b, int B, hipStream_t st) {
  hipLaunchKernelGGL(c51_loss_kernel, dim3((B + 3) / 4), dim3(256), 0, st, hc, ldh, hb, A, Z, act, m, 1.0f / (float)B,
                     dh, loss_b, logit_b, B);
}

void embed_bwd(const float* dfeat, int ldf, int off, const float* emb, int D, const int* task, int B, int T,
               float* demb, hipStream_t st) {
  hipLaunchKernelGGL(embed_bwd_kernel, dim3(T), dim3(64), 0, st, dfeat, ldf, off, emb, D, task, B, demb);
}

void enc_grad(const float* dfeat, int ldf, const float* enc, int nenc, float* denc, int B, hipStream_t st) {
  hipLaunchKernelGGL(enc_grad_kernel, dim3(blocks((long long)B * nenc)), dim3(256), 0, st, dfeat, ldf, enc, nenc, denc,
                     B);
}

int adamw(float* p, float* mu, float* nu, const float* g, float* tgt, long long n, float lr, float b1, float b2,
          float eps, float wd, float tau, int count, float* part, int max_blocks, hipStream_t st) {
  const int G = (int)std::min<long long>(max_blocks, std::max<long long>(1, (n + 255) / 256));
  hipLaunchKernelGGL(adamw_kernel, dim3(G), dim3(256), 0, st, p, mu, nu, g, tgt, n, lr, b1, b2, eps, wd, tau, count,
                     part);
  return G;
}

void drq_logs(const float* part, int G, const float* loss_b, const float* logit_b, int B, int Z, float* logs,
              hipStream_t st) {
  hipLaunchKernelGGL(drq_logs_kernel, dim3(1), dim3(256), 0, st, part, G, loss_b, logit_b, B, Z, logs);
}


// ------------------------------------------------------------------ compute_weights launchers
void flax_gather(const float* g, const long long* map, int entries, long long max_n, float* out, hipStream_t st) {
  const unsigned gx = (unsigned)std::min<long long>((max_n + 255) / 256, 4096);
  hipLaunchKernelGGL(flax_gather_kernel, dim3(gx, entries), dim3(256), 0, st, g, map, out);
}

int jl_splits(long long P, int D) {
  const long long jb = (D + 255) / 256;
  long long s = (2048 + jb - 1) / jb;  // >= 2048 workgroups over the 256 CUs
  s = std::min<long long>(s, (P + JL_K - 1) / JL_K);
  return (int)std::max<long long>(s, 1);
}

long long jl_part_floats(long long P, int D) { return (long long)jl_splits(P, D) * JL_T * D; }

int jl_max_tasks() { return JL_T; }

void jl_project(const float* G, long long ldg, int T, long long P, int D, long long chunk, int seed, float* part,
                float* out, long long ldo, hipStream_t st) {
  const int splits = jl_splits(P, D);
  long long kper = (P + splits - 1) / splits;
  kper = (kper + JL_K - 1) / JL_K * JL_K;
  const int used = (int)((P + kper - 1) / kper);
  hipLaunchKernelGGL(jl_project_kernel, dim3((D + 255) / 256, used), dim3(256), 0, st, G, ldg, T, P, D, chunk, seed,
                     kper, part);
  const long long n = (long long)T * D;
  hipLaunchKernelGGL(jl_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, part, used, T, D,
                     sqrtf((float)D), out, ldo);
}

}  // namespace drq
}  // namespace mtsac
