// Small fused elementwise / reduction kernels.
//
// act_bwd:  dz = dh * dropout_mask / keep * act'(z), plus colsum(dz) into an fp32
//           bias-grad.  Used where the producer of dh cannot fold
//           it into its GEMM epilogue -- at a pipeline-stage boundary, where dh
//           arrives over xGMI from the next stage.
// metrics_fold: running[0:4] += slot[0:4]; slot = 0   (data_paral.py:234-236)
#include "common.h"

namespace jdt {

__global__ void __launch_bounds__(256) act_bwd_kernel(const bf16_t* __restrict__ dh, const bf16_t* __restrict__ z,
                                                      int act, float keep_prob, unsigned long long seed,
                                                      unsigned long long offset, const int* step_ptr,
                                                      const unsigned long long* seed_ptr, int M, int N,
                                                      int rows_per_block, bf16_t* __restrict__ dz,
                                                      float* __restrict__ dbias) {
  const int col = blockIdx.x * 256 + threadIdx.x;
  if (col >= N) return;
  const int r0 = blockIdx.y * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  const bool drop = keep_prob < 1.f;
  const float inv_keep = drop ? 1.f / keep_prob : 1.f;
  const unsigned long long doff = offset + (step_ptr ? ((unsigned long long)(unsigned)step_ptr[0] << 32) : 0ull);
  if (seed_ptr) seed = seed_ptr[0];
  float csum = 0.f;
  u32x4 dbits = {0u, 0u, 0u, 0u};
  for (int r = r0; r < r1; ++r) {  // r0 is a multiple of 4: refresh the Philox bits per 4-row group
    const long i = (long)r * N + col;
    if (drop && (r & 3) == 0) dbits = dropout_bits(seed, doff, dropout_group(0, r, col, M, N));
    float v = bf2f(dh[i]);
    if (z) v *= act_grad(act, bf2f(z[i]));
    if (drop) v = keep_word(dbits, r & 3, keep_prob) ? v * inv_keep : 0.f;
    const bf16_t o = f2bf(v);
    dz[i] = o;
    csum += bf2f(o);
  }
  if (dbias) atomicAdd(dbias + col, csum);
}

__global__ void metrics_fold_kernel(float* running, float* slot, int n) {
  const int i = threadIdx.x;
  if (i < n) { running[i] += slot[i]; slot[i] = 0.f; }
}

}  // namespace jdt
using namespace jdt;

JDT_API int jdt_act_bwd(const void* dh, const void* z, int act, float keep_prob, unsigned long long seed,
                        unsigned long long offset, const int* step_ptr, const unsigned long long* seed_ptr, int M,
                        int N, void* dz, float* dbias, void* stream) {
  if (M <= 0 || N <= 0) return 0;
  const int rpb = 32;
  dim3 grid((N + 255) / 256, (M + rpb - 1) / rpb);
  hipLaunchKernelGGL(act_bwd_kernel, grid, dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const bf16_t*>(dh), static_cast<const bf16_t*>(z), act, keep_prob, seed, offset,
                     step_ptr, seed_ptr, M, N, rpb, static_cast<bf16_t*>(dz), dbias);
  return HIP_LAUNCH_CHECK();
}

JDT_API int jdt_metrics_fold(float* running, float* slot, int n, void* stream) {
  hipLaunchKernelGGL(metrics_fold_kernel, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream), running, slot, n);
  return HIP_LAUNCH_CHECK();
}
