// Fused softmax cross-entropy with integer labels: forward, backward and the
// (sum, count) metrics in one pass over the logits.
//
// Reference semantics (data_paral.py:171-189): logits are cast to fp32,
// loss = optax.softmax_cross_entropy_with_integer_labels, accuracy =
// argmax == label, metrics {"loss": (sum, n), "accuracy": (correct, n)},
// returned loss = mean.  Here the gradient of `grad_scale * sum(loss)` is
// written directly (grad_scale = 1 / rows for a mean), so the logits never
// make a second trip through HBM, and the metrics go to a device-resident
// fp32[4] accumulator with one atomic per workgroup.
//
// One wave per row (64-wide online max/sum over the classes); rows with
// label < 0 are ignored (ignore_index) and contribute zero gradient.
#include "common.h"

namespace jdt {

template <bool F32>
__device__ __forceinline__ float ld_logit(const void* p, long i) {
  return F32 ? static_cast<const float*>(p)[i] : bf2f(static_cast<const bf16_t*>(p)[i]);
}

template <bool F32>
__global__ void __launch_bounds__(256) xent_kernel(const void* logits, long ld, const int* labels, int M, int C,
                                                   float grad_scale, bf16_t* dlogits, long ldd, float* dbias,
                                                   float* metrics, float* row_loss) {
  __shared__ float red[4][4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int row = blockIdx.x * 4 + w;
  float l_sum = 0.f, n_valid = 0.f, n_correct = 0.f;
  if (row < M) {
    const int label = labels[row];
    const long base = (long)row * ld;
    // pass 1: online max / sum-exp and argmax
    float mx = -INFINITY, s = 0.f, best = -INFINITY;
    int besti = 0x7fffffff;
    for (int c = lane; c < C; c += 64) {
      const float z = ld_logit<F32>(logits, base + c);
      if (z > best) { best = z; besti = c; }
      const float nm = fmaxf(mx, z);
      s = s * __expf(mx - nm) + __expf(z - nm);
      mx = nm;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float omx = __shfl_xor(mx, o, 64), os = __shfl_xor(s, o, 64);
      const float nm = fmaxf(mx, omx);
      s = (nm == -INFINITY) ? 0.f : s * __expf(mx - nm) + os * __expf(omx - nm);
      mx = nm;
      const float ob = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(besti, o, 64);
      if (ob > best || (ob == best && oi < besti)) { best = ob; besti = oi; }
    }
    const float lse = mx + __logf(s);
    const bool valid = label >= 0 && label < C;
    const float zl = valid ? ld_logit<F32>(logits, base + label) : 0.f;
    const float loss = valid ? lse - zl : 0.f;
    if (row_loss && lane == 0) row_loss[row] = loss;
    if (valid) { l_sum = loss; n_valid = 1.f; n_correct = (besti == label) ? 1.f : 0.f; }
    // pass 2: gradient (softmax - onehot) * grad_scale
    if (dlogits) {
      for (int c = lane; c < C; c += 64) {
        float gval = 0.f;
        if (valid) {
          const float p = __expf(ld_logit<F32>(logits, base + c) - lse);
          gval = (p - (c == label ? 1.f : 0.f)) * grad_scale;
        }
        const bf16_t gb = f2bf(gval);
        dlogits[(long)row * ldd + c] = gb;
        if (dbias && valid) atomicAdd(dbias + c, bf2f(gb));
      }
    }
  }
  if (metrics) {
    if (lane == 0) { red[w][0] = l_sum; red[w][1] = n_valid; red[w][2] = n_correct; }
    __syncthreads();
    if (threadIdx.x == 0) {
      float a = 0.f, b = 0.f, c = 0.f;
      for (int i = 0; i < 4; ++i) { a += red[i][0]; b += red[i][1]; c += red[i][2]; }
      if (b > 0.f) {
        atomicAdd(metrics + 0, a); atomicAdd(metrics + 1, b);
        atomicAdd(metrics + 2, c); atomicAdd(metrics + 3, b);
      }
    }
  }
}

}  // namespace jdt
using namespace jdt;

JDT_API int jdt_xent(const void* logits, int logits_f32, long ld, const int* labels, int M, int C, float grad_scale,
                     void* dlogits, long ldd, float* dbias, float* metrics, float* row_loss, void* stream) {
  if (M <= 0) return 0;
  dim3 grid((M + 3) / 4);
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (logits_f32)
    hipLaunchKernelGGL(xent_kernel<true>, grid, dim3(256), 0, st, logits, ld, labels, M, C, grad_scale,
                       static_cast<bf16_t*>(dlogits), ldd, dbias, metrics, row_loss);
  else
    hipLaunchKernelGGL(xent_kernel<false>, grid, dim3(256), 0, st, logits, ld, labels, M, C, grad_scale,
                       static_cast<bf16_t*>(dlogits), ldd, dbias, metrics, row_loss);
  return HIP_LAUNCH_CHECK();
}
