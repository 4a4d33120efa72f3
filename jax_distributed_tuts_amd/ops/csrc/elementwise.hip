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

// metrics_fold_slab: running[0:4] += slot[0:4] + (sum of the slab's rows as {loss, n,
// correct, n}); slot = 0, every slab row = 0; then (step non-null) the device step += 1 --
// the step-end fold of a pass whose CE wrote per-workgroup metric rows (jdt_xent_slab) and
// whose AdamW ranges ran without advancing the step, beside the W pass that also reads it
// Latency-bound (one workgroup, 16 KB): every load -- FOLD_U slab rows per thread, the
// running / slot values and the step -- is issued before the first use (one memory round
// trip; the per-row load/store loop was one per 256 rows: 4.6 us per step in the LM), the
// wave sums are DPP moves and the 4 waves meet in LDS behind one barrier.
constexpr int FOLD_U = 4;
__global__ void __launch_bounds__(256) metrics_fold_slab_kernel(float* running, float* slot, int n,
                                                                float4* __restrict__ slab, int cap, int* step) {
  __shared__ float red[4][3];
  const int t = threadIdx.x, w = t >> 6;
  const float run = t < n ? running[t] : 0.f, sl = t < n ? slot[t] : 0.f;
  const int sv = (t == 0 && step) ? step[0] : 0;
  float a = 0.f, b = 0.f, c = 0.f;
  for (int i0 = 0; i0 < cap; i0 += 256 * FOLD_U) {
    float4 r[FOLD_U];
#pragma unroll
    for (int u = 0; u < FOLD_U; ++u) {
      const int i = i0 + u * 256 + t;
      r[u] = i < cap ? slab[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < FOLD_U; ++u) {
      const int i = i0 + u * 256 + t;
      a += r[u].x; b += r[u].y; c += r[u].z;
      if (i < cap) slab[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  a = wave_sum_dpp(a); b = wave_sum_dpp(b); c = wave_sum_dpp(c);
  if ((t & 63) == 0) { red[w][0] = a; red[w][1] = b; red[w][2] = c; }
  __syncthreads();
  if (t < n) {
    const int k = t == 0 ? 0 : (t == 2 ? 2 : 1);
    const float add = t < 4 ? (red[0][k] + red[1][k]) + (red[2][k] + red[3][k]) : 0.f;
    running[t] = run + (sl + add);
    slot[t] = 0.f;
  }
  if (t == 0 && step) step[0] = sv + 1;
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

JDT_API int jdt_metrics_fold_slab(float* running, float* slot, int n, float* slab, int cap, int* step, void* stream) {
  if (n > 256 || cap < 0 || (reinterpret_cast<uintptr_t>(slab) & 15)) return -2;
  hipLaunchKernelGGL(metrics_fold_slab_kernel, dim3(1), dim3(256), 0, static_cast<hipStream_t>(stream), running, slot,
                     n, reinterpret_cast<float4*>(slab), cap, step);
  return HIP_LAUNCH_CHECK();
}
