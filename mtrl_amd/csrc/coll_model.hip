// coll_model.hip -- the modelled trunk-gradient collective (include/mtsac_debug.h,
// mtsac_debug_set_collective_model): what one rank's all-reduce of a bucket costs on an N-GPU node,
// issued at the RCCL points on the collective stream of a ONE-GPU run.
//
// A ring all-reduce moves 2 (N - 1) / N of the bucket through each rank's busiest link, so the
// modelled time is that many bytes over an assumed bus bandwidth; the kernel holds `blocks`
// workgroups (the CUs an RCCL all-reduce keeps busy) for that long, timed by the 100 MHz constant
// clock (s_memrealtime: DVFS does not stretch it).  The data are left as they are: a one-rank
// reduction is the identity.  With `poison` the bucket is first saved and overwritten with NaN and
// restored only after the delay, so a consumer that reads the bucket before the collective is done
// (a missing stream edge) turns the step's results into NaN instead of silently reading the
// pre-reduction values.
#include "kernels.h"

namespace mtsac {

namespace {

__global__ void cm_delay_kernel(unsigned long long ticks) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

__global__ void cm_poison_kernel(float* __restrict__ buf, float* __restrict__ shadow, long long n) {
  const float nan = __builtin_nanf("");
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    shadow[i] = buf[i];
    buf[i] = nan;
  }
}

__global__ void cm_restore_kernel(float* __restrict__ buf, const float* __restrict__ shadow, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    buf[i] = shadow[i];
}

}  // namespace

double coll_model_us(long long bytes, int nranks, double bus_gbps) {
  if (nranks <= 1 || bus_gbps <= 0.0) return 0.0;
  return 2.0 * (nranks - 1) / nranks * (double)bytes / (bus_gbps * 1e3);  // bytes / (GB/s) = ns
}

// scale: the share of an all-reduce's link time the collective takes (0.5: a reduce-scatter or an
// all-gather, (N - 1) / N of the bucket each)
void coll_model_allreduce(float* buf, long long count, int nranks, double bus_gbps, int blocks, float* shadow,
                          hipStream_t st, double scale) {
  const int g = (int)std::min<long long>(1024, std::max<long long>(1, (count + 255) / 256));
  if (shadow) hipLaunchKernelGGL(cm_poison_kernel, dim3(g), dim3(256), 0, st, buf, shadow, count);
  const double us = scale * coll_model_us(count * 4, nranks, bus_gbps);
  const unsigned long long ticks = (unsigned long long)(us * 100.0 + 0.5);  // 100 MHz: 10 ns per tick
  if (ticks > 0) hipLaunchKernelGGL(cm_delay_kernel, dim3(std::max(1, blocks)), dim3(64), 0, st, ticks);
  if (shadow) hipLaunchKernelGGL(cm_restore_kernel, dim3(g), dim3(256), 0, st, buf, shadow, count);
}

}  // namespace mtsac
