// Fused optimizer steps over one flat fp32 parameter buffer.
//
// optax.adamw defaults (data_paral.py:106-108, param_sharding.py:235-237):
//   b1 0.9, b2 0.999, eps 1e-8 (outside the sqrt), weight_decay 1e-4 applied to
//   every leaf (mask None), bias correction with the step count.
// In one pass per element:
//   g   = grad * grad_scale            (1/n_minibatches * 1/n_devices folded here)
//   m,v = moments ; p -= lr * (m_hat / (sqrt(v_hat) + eps) + wd * p)
//   shadow_bf16 = bf16(p)             (the compute copy every GEMM reads)
//   grad = 0                           (ready for the next step's beta=1 accumulation)
// The step counter lives on the device so the kernel is replayable from a
// hipGraph: every workgroup reads it, and the workgroup that takes the last
// arrival ticket advances it and re-arms the ticket for the next launch.
#include "common.h"

namespace jdt {

__device__ __forceinline__ void finish_ticket(int* step, unsigned* ticket) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = atomicAdd(ticket, 1u);
    if (t == gridDim.x - 1) {
      step[0] = step[0] + 1;
      __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

constexpr int AW_U = 4;

// AdamW on U float4 groups at float4 indices idx[u] (loads first, then math, then the
// stores of the groups whose logical index q0 + u * stride is < n4)
template <int U>
__device__ __forceinline__ void adam_rows(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                          float* __restrict__ v, bf16_t* __restrict__ shadow, const long (&idx)[U],
                                          long q0, long stride, long n4, float lr, float b1, float b2, float eps,
                                          float wd, float grad_scale, float rbc1, float rbc2, int zero_grad) {
  float4 pp[U], gg[U], mm[U], vv[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    pp[u] = reinterpret_cast<const float4*>(p)[idx[u]];
    gg[u] = reinterpret_cast<const float4*>(g)[idx[u]];
    mm[u] = reinterpret_cast<const float4*>(m)[idx[u]];
    vv[u] = reinterpret_cast<const float4*>(v)[idx[u]];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    float* pe = &pp[u].x; float* ge = &gg[u].x; float* me = &mm[u].x; float* ve = &vv[u].x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gr = ge[k] * grad_scale;
      me[k] = b1 * me[k] + (1.f - b1) * gr;
      ve[k] = b2 * ve[k] + (1.f - b2) * gr * gr;
      const float upd = (me[k] * rbc1) / (sqrtf(ve[k] * rbc2) + eps) + wd * pe[k];
      pe[k] -= lr * upd;
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (q0 + u * stride >= n4) break;   // uniform for all but the last round
    const long i = idx[u];
    reinterpret_cast<float4*>(p)[i] = pp[u];
    reinterpret_cast<float4*>(m)[i] = mm[u];
    reinterpret_cast<float4*>(v)[i] = vv[u];
    if (zero_grad) reinterpret_cast<float4*>(g)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (shadow) {
      uint2 sh;
      sh.x = (unsigned)f2bf(pp[u].x) | ((unsigned)f2bf(pp[u].y) << 16);
      sh.y = (unsigned)f2bf(pp[u].z) | ((unsigned)f2bf(pp[u].w) << 16);
      reinterpret_cast<uint2*>(shadow)[i] = sh;
    }
  }
}

__global__ void __launch_bounds__(256) adamw_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                                                    float* __restrict__ v, bf16_t* __restrict__ shadow, long n,
                                                    float lr, float b1, float b2, float eps, float wd, float grad_scale,
                                                    int* step, unsigned* ticket, int zero_grad) {
  const int t = step[0] + 1;
  const float bc1 = 1.f - powf(b1, (float)t), bc2 = 1.f - powf(b2, (float)t);
  const float rbc1 = 1.f / bc1, rbc2 = 1.f / bc2;
  const long n4 = n / 4;
  const long stride = (long)gridDim.x * blockDim.x;
  // AW_U float4 per thread per round, every load issued before any use (clamped
  // indices, no branch around a load): a round trip per AW_U elements instead of one
  // per element, so a one-workgroup-per-CU grid still streams at HBM rate
  for (long q0 = (long)blockIdx.x * blockDim.x + threadIdx.x; q0 < n4; q0 += AW_U * stride) {
    long idx[AW_U];
#pragma unroll
    for (int u = 0; u < AW_U; ++u) idx[u] = min(q0 + u * stride, n4 - 1);
    adam_rows<AW_U>(p, g, m, v, shadow, idx, q0, stride, n4, lr, b1, b2, eps, wd, grad_scale, rbc1, rbc2, zero_grad);
  }
  // tail
  for (long i = n4 * 4 + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float gr = g[i] * grad_scale;
    const float mi = b1 * m[i] + (1.f - b1) * gr;
    const float vi = b2 * v[i] + (1.f - b2) * gr * gr;
    m[i] = mi; v[i] = vi;
    const float pi = p[i] - lr * ((mi * rbc1) / (sqrtf(vi * rbc2) + eps) + wd * p[i]);
    p[i] = pi;
    if (zero_grad) g[i] = 0.f;
    if (shadow) shadow[i] = f2bf(pi);
  }
  // ticket null: one range of a step split over several launches (the caller advances
  // the step once every range has read it, OverlappedAdamW)
  if (ticket) finish_ticket(step, ticket);
}

// AdamW over a list of ranges of the flat buffers (the parameters whose update did
// NOT ride in a weight-gradient GEMM epilogue: biases, LayerNorm, embeddings) in ONE
// launch; ranges are multiples of 4 elements (FlatParams views are 64-aligned and
// padded), prefix[r] = elements before range r.  Advances the step counter once.
__global__ void __launch_bounds__(256) adamw_ranges_kernel(float* __restrict__ p, float* __restrict__ g,
                                                           float* __restrict__ m, float* __restrict__ v,
                                                           bf16_t* __restrict__ shadow, const long* __restrict__ start,
                                                           const long* __restrict__ prefix, int nr, long total,
                                                           float lr, float b1, float b2, float eps, float wd,
                                                           float grad_scale, int* step, unsigned* ticket) {
  const int t = step[0] + 1;
  const float rbc1 = 1.f / (1.f - powf(b1, (float)t)), rbc2 = 1.f / (1.f - powf(b2, (float)t));
  const long n4 = total / 4;
  const long stride = (long)gridDim.x * blockDim.x;
  for (long q0 = (long)blockIdx.x * blockDim.x + threadIdx.x; q0 < n4; q0 += AW_U * stride) {
    long idx[AW_U];
#pragma unroll
    for (int u = 0; u < AW_U; ++u) {
      const long e = 4 * min(q0 + u * stride, n4 - 1);
      int lo = 0, hi = nr - 1;   // last range with prefix <= e
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (prefix[mid] <= e) lo = mid; else hi = mid - 1;
      }
      idx[u] = (start[lo] + (e - prefix[lo])) >> 2;   // float4 index
    }
    adam_rows<AW_U>(p, g, m, v, shadow, idx, q0, stride, n4, lr, b1, b2, eps, wd, grad_scale, rbc1, rbc2, 1);
  }
  // ticket null: the ranges run beside other readers of the step (the LM's W pass on the
  // main stream); the caller advances the step after both (jdt_metrics_fold_slab)
  if (ticket) finish_ticket(step, ticket);
}

// SGD (+ optional heavy-ball momentum and decoupled weight decay)
__global__ void __launch_bounds__(256) sgd_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ buf,
                                                  bf16_t* __restrict__ shadow, long n, float lr, float momentum,
                                                  float wd, float grad_scale, int* step, unsigned* ticket,
                                                  int zero_grad) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float gr = g[i] * grad_scale + wd * p[i];
    if (buf) { gr = momentum * buf[i] + gr; buf[i] = gr; }
    const float pi = p[i] - lr * gr;
    p[i] = pi;
    if (zero_grad) g[i] = 0.f;
    if (shadow) shadow[i] = f2bf(pi);
  }
  if (step) finish_ticket(step, ticket);
}

__global__ void cast_f32_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, long n) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) y[i] = f2bf(x[i]);
}

__global__ void scale_kernel(float* __restrict__ x, long n, float s) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) x[i] *= s;
}

static int grid_for(long n, int per_thread, int cap = 2048) {
  long b = (n / per_thread + 255) / 256;
  if (b < 1) b = 1;
  if (b > cap) b = cap;  // grid-stride beyond that
  return (int)b;
}

// Kernels that advance the device step counter end with one same-address
// arrival ticket per workgroup; those atomics serialise, so those kernels run
// at most one workgroup per CU and grid-stride over the rest.
constexpr int kTicketGrid = 256;
// (Round 2 grew the grid to 2048 workgroups above ~1M elements because a 256-workgroup
// grid-stride loop was latency-bound; but 2048 same-address tickets serialise at
// ~12.7 ns each = 26 us, most of the transformer's 23 us AdamW launch.  The AdamW loops
// now keep AW_U groups of loads in flight per thread instead, so one workgroup per CU
// streams at HBM rate and the ticket chain is 256 long.)
static int ticket_grid(long n, int per_thread) { return grid_for(n, per_thread, kTicketGrid); }

}  // namespace jdt
using namespace jdt;

JDT_API int jdt_adamw(float* p, float* g, float* m, float* v, void* shadow, long n, float lr, float b1, float b2,
                      float eps, float wd, float grad_scale, int* step, unsigned* ticket, int zero_grad,
                      void* stream) {
  if (n <= 0) return 0;
  if ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(m) |
       reinterpret_cast<uintptr_t>(v)) & 15) return -2;
  if (shadow && (reinterpret_cast<uintptr_t>(shadow) & 7)) return -2;
  hipLaunchKernelGGL(adamw_kernel, dim3(ticket_grid(n, 4)), dim3(256), 0, static_cast<hipStream_t>(stream), p, g, m, v,
                     static_cast<bf16_t*>(shadow), n, lr, b1, b2, eps, wd, grad_scale, step, ticket, zero_grad);
  return HIP_LAUNCH_CHECK();
}

// ranges: device int64 start[nr] (element offsets, % 4 == 0), prefix[nr] (exclusive sums of
// the lengths, each % 4 == 0); total = sum of the lengths.  Needs step; ticket null = the
// step is NOT advanced (the caller does it once every reader of the step has run).
JDT_API int jdt_adamw_ranges(float* p, float* g, float* m, float* v, void* shadow, const long* start,
                             const long* prefix, int nr, long total, float lr, float b1, float b2, float eps, float wd,
                             float grad_scale, int* step, unsigned* ticket, void* stream) {
  if (nr <= 0 || total <= 0 || (total & 3) || !step || !shadow) return -2;
  if ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(m) |
       reinterpret_cast<uintptr_t>(v)) & 15) return -2;
  if (reinterpret_cast<uintptr_t>(shadow) & 7) return -2;
  hipLaunchKernelGGL(adamw_ranges_kernel, dim3(ticket_grid(total, 4)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     p, g, m, v, static_cast<bf16_t*>(shadow), start, prefix, nr, total, lr, b1, b2, eps, wd,
                     grad_scale, step, ticket);
  return HIP_LAUNCH_CHECK();
}

JDT_API int jdt_sgd(float* p, float* g, float* buf, void* shadow, long n, float lr, float momentum, float wd,
                    float grad_scale, int* step, unsigned* ticket, int zero_grad, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(sgd_kernel, dim3(step ? ticket_grid(n, 1) : grid_for(n, 1)), dim3(256), 0, static_cast<hipStream_t>(stream), p, g, buf,
                     static_cast<bf16_t*>(shadow), n, lr, momentum, wd, grad_scale, step, ticket, zero_grad);
  return HIP_LAUNCH_CHECK();
}

JDT_API int jdt_cast_f32_bf16(const float* x, void* y, long n, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(grid_for(n, 1)), dim3(256), 0, static_cast<hipStream_t>(stream), x,
                     static_cast<bf16_t*>(y), n);
  return HIP_LAUNCH_CHECK();
}

JDT_API int jdt_scale(float* x, long n, float s, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(scale_kernel, dim3(grid_for(n, 1)), dim3(256), 0, static_cast<hipStream_t>(stream), x, n, s);
  return HIP_LAUNCH_CHECK();
}
