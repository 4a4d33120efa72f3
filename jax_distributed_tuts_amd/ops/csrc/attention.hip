// Transformer helpers: causal row-softmax fwd/bwd for attention, token +
// position embedding fwd/bwd, and a bias-gradient column sum.
//
// Attention is composed as  S = alpha * Q K^T  (MFMA GEMM, 2-level batch over
// (batch, head) reading q/k/v in place from the fused [T, 3d] QKV projection),
// P = softmax_causal(S) (this file), O = P V (MFMA GEMM writing [T, d] in place).
// Backward: dP = dO V^T, dS = P * (dP - rowsum(P * dP)) (this file),
// dQ = alpha dS K, dK = alpha dS^T Q, dV = P^T dO -- all on the same GEMM kernel.
#include "common.h"

namespace jdt {

// one wave per row, row length Sk <= 64 * 32
__global__ void __launch_bounds__(256) attn_softmax_fwd_kernel(const float* __restrict__ S, bf16_t* __restrict__ P,
                                                              int rows, int Sq, int Sk, int causal) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int q = (int)(row % Sq);
  const int lim = causal ? min(Sk, q + 1 + (Sk - Sq)) : Sk;  // keys [0, lim) visible
  const float* s = S + row * Sk;
  float mx = -INFINITY;
  for (int k = lane; k < lim; k += 64) mx = fmaxf(mx, s[k]);
  mx = wave_max(mx);
  float sum = 0.f;
  for (int k = lane; k < lim; k += 64) sum += __expf(s[k] - mx);
  sum = wave_sum(sum);
  const float inv = 1.f / sum;
  bf16_t* p = P + row * Sk;
  for (int k = lane; k < Sk; k += 64) p[k] = k < lim ? f2bf(__expf(s[k] - mx) * inv) : (bf16_t)0;
}

__global__ void __launch_bounds__(256) attn_softmax_bwd_kernel(const bf16_t* __restrict__ P, const float* __restrict__ dP,
                                                              bf16_t* __restrict__ dS, int rows, int Sk) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const bf16_t* p = P + row * Sk;
  const float* dp = dP + row * Sk;
  float dot = 0.f;
  for (int k = lane; k < Sk; k += 64) dot += bf2f(p[k]) * dp[k];
  dot = wave_sum(dot);
  bf16_t* ds = dS + row * Sk;
  for (int k = lane; k < Sk; k += 64) ds[k] = f2bf(bf2f(p[k]) * (dp[k] - dot));
}

__global__ void __launch_bounds__(256) embed_fwd_kernel(const int* __restrict__ tok, const bf16_t* __restrict__ wte,
                                                       const bf16_t* __restrict__ wpe, bf16_t* __restrict__ out,
                                                       int T, int S, int d) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;  // one thread per 8 columns
  const int per_row = d / 8;
  if (i >= (long)T * per_row) return;
  const int t = (int)(i / per_row), c = (int)(i % per_row) * 8;
  const int v = tok[t], pos = t % S;
  const u32x4 a = *reinterpret_cast<const u32x4*>(wte + (long)v * d + c);
  const u32x4 b = *reinterpret_cast<const u32x4*>(wpe + (long)pos * d + c);
  *reinterpret_cast<u32x4*>(out + (long)t * d + c) = bf16x8_add(a, b);
}

__global__ void __launch_bounds__(256) embed_bwd_kernel(const bf16_t* __restrict__ dout, const int* __restrict__ tok,
                                                       float* __restrict__ dwte, float* __restrict__ dwpe, int T, int S,
                                                       int d) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)T * d) return;
  const int t = (int)(i / d), c = (int)(i % d);
  const float g = bf2f(dout[i]);
  atomicAdd(dwte + (long)tok[t] * d + c, g);
  // the position table's gradient: a thread of the first sequence sums its (position,
  // column) over every sequence in order and adds once -- T / S times fewer atomics than
  // one per token (each position row took T / S same-address adds)
  if (dwpe && t < S) {
    float sp = g;
    for (int q = t + S; q < T; q += S) sp += bf2f(dout[(long)q * d + c]);
    atomicAdd(dwpe + (long)t * d + c, sp);
  }
}

// out[c] += sum_r x[r, c] (bias gradients).  A lane owns 8 adjacent columns
// (one 16-byte load per row), a wave CS_RPW rows whose loads are all issued
// before the first add, the 4 waves of a workgroup are summed in LDS, and one
// fp32 atomic per column per workgroup goes to the output.
constexpr int CS_RPW = 8;

__global__ void __launch_bounds__(256) colsum_kernel(const bf16_t* __restrict__ x, long ld, int M, int N,
                                                    float* __restrict__ out) {
  __shared__ float part[4][512];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = blockIdx.x * 512 + lane * 8;
  const int r0 = (blockIdx.y * 4 + w) * CS_RPW;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (col < N) {
    u32x4 v[CS_RPW];
#pragma unroll
    for (int i = 0; i < CS_RPW; ++i) {
      v[i] = (u32x4){0u, 0u, 0u, 0u};
      if (r0 + i < M) v[i] = *reinterpret_cast<const u32x4*>(x + (long)(r0 + i) * ld + col);
    }
#pragma unroll
    for (int i = 0; i < CS_RPW; ++i) {
      const unsigned wv[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += bf2f((bf16_t)((wv[j >> 1] >> (16 * (j & 1))) & 0xffffu));
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) part[w][lane * 8 + j] = s[j];
  __syncthreads();
  for (int c = threadIdx.x; c < 512; c += 256) {
    const int gc = blockIdx.x * 512 + c;
    if (gc < N) atomicAdd(out + gc, part[0][c] + part[1][c] + part[2][c] + part[3][c]);
  }
}

}  // namespace jdt
using namespace jdt;

JDT_API int jdt_attn_softmax_fwd(const float* S, void* P, int rows, int Sq, int Sk, int causal, void* stream) {
  hipLaunchKernelGGL(attn_softmax_fwd_kernel, dim3((rows + 3) / 4), dim3(256), 0, static_cast<hipStream_t>(stream), S,
                     static_cast<bf16_t*>(P), rows, Sq, Sk, causal);
  return HIP_LAUNCH_CHECK();
}

JDT_API int jdt_attn_softmax_bwd(const void* P, const float* dP, void* dS, int rows, int Sk, void* stream) {
  hipLaunchKernelGGL(attn_softmax_bwd_kernel, dim3((rows + 3) / 4), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const bf16_t*>(P), dP, static_cast<bf16_t*>(dS), rows, Sk);
  return HIP_LAUNCH_CHECK();
}

JDT_API int jdt_embed_fwd(const int* tok, const void* wte, const void* wpe, void* out, int T, int S, int d,
                          void* stream) {
  if (d % 8) return -3;
  const long n = (long)T * (d / 8);
  hipLaunchKernelGGL(embed_fwd_kernel, dim3((n + 255) / 256), dim3(256), 0, static_cast<hipStream_t>(stream), tok,
                     static_cast<const bf16_t*>(wte), static_cast<const bf16_t*>(wpe), static_cast<bf16_t*>(out), T,
                     S, d);
  return HIP_LAUNCH_CHECK();
}

JDT_API int jdt_embed_bwd(const void* dout, const int* tok, float* dwte, float* dwpe, int T, int S, int d,
                          void* stream) {
  const long n = (long)T * d;
  hipLaunchKernelGGL(embed_bwd_kernel, dim3((n + 255) / 256), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const bf16_t*>(dout), tok, dwte, dwpe, T, S, d);
  return HIP_LAUNCH_CHECK();
}

JDT_API int jdt_colsum(const void* x, long ld, int M, int N, float* out, void* stream) {
  if (M <= 0 || N <= 0) return 0;
  if ((N & 7) || (ld & 7) || (reinterpret_cast<uintptr_t>(x) & 15)) return -3;
  dim3 grid((N + 511) / 512, (M + 4 * CS_RPW - 1) / (4 * CS_RPW));
  hipLaunchKernelGGL(colsum_kernel, grid, dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const bf16_t*>(x), ld, M, N, out);
  return HIP_LAUNCH_CHECK();
}
