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

// Metrics epilogue shared by both kernels: the workgroup's (loss, valid, correct)
// sums -> metrics[0..3] += (loss, n, correct, n), one atomic per slot.  (A
// two-level ticket tree instead of the same-address atomics measured slower: its
// latency chain of two device-scope tickets and two row loads costs ~6 us against
// the atomics' serialisation, tools/bench_xent.py; fewer, longer workgroups are the
// cheaper fix, see rpw.)
__device__ __forceinline__ void xent_metrics_fold(float (*red)[4], int w, int lane, float l_sum, float n_valid,
                                                  float n_correct, float* metrics) {
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
  if (metrics) xent_metrics_fold(red, w, lane, l_sum, n_valid, n_correct, metrics);
}


// Wide-vocabulary variant (bf16 logits, C % 8 == 0, C <= 512 * NV): a lane owns
// NV chunks of 8 adjacent classes, so a row is NV 16-byte loads per lane held
// in registers -- max, sum-exp, argmax and the gradient all come from those
// registers (one HBM read, one write).  A wave walks `rpw` rows and keeps its
// bias-gradient partials in registers; the 4 waves are summed in LDS and each
// workgroup adds one fp32 atomic per class.
template <int NV>
__global__ void __launch_bounds__(256) xent_vec_kernel(const bf16_t* __restrict__ logits, long ld,
                                                       const int* __restrict__ labels, int M, int C, int rpw,
                                                       float grad_scale, bf16_t* __restrict__ dlogits, long ldd,
                                                       float* __restrict__ dbias, float* __restrict__ metrics,
                                                       float* __restrict__ row_loss, float4* __restrict__ mslab) {
  __shared__ float red[4][4];
  __shared__ float part[4][512 * NV];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float l_sum = 0.f, n_valid = 0.f, n_correct = 0.f;
  float db[NV][8];
#pragma unroll
  for (int k = 0; k < NV; ++k)
#pragma unroll
    for (int j = 0; j < 8; ++j) db[k][j] = 0.f;
  // row blocks [x G/8, (x+1) G/8) on XCD x: the rows the head GEMM's tile map wrote there and
  // its input-gradient GEMM reads there (gemm_dma_kernel: contiguous tile ranges per XCD)
  const int G = gridDim.x, blk = (G & 7) ? blockIdx.x : (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  const int r0 = (blk * 4 + w) * rpw;
  for (int row = r0; row < min(M, r0 + rpw); ++row) {
    const int label = labels[row];
    const bool valid = label >= 0 && label < C;
    float z[NV][8];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c0 = (k * 64 + lane) * 8;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (c0 < C) v = *reinterpret_cast<const u32x4*>(logits + (long)row * ld + c0);
      const unsigned wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 8; ++j)
        z[k][j] = c0 < C ? bf2f((bf16_t)((wv[j >> 1] >> (16 * (j & 1))) & 0xffffu)) : -INFINITY;
    }
    float mx = -INFINITY;
    int besti = 0x7fffffff;
#pragma unroll
    for (int k = 0; k < NV; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (z[k][j] > mx) { mx = z[k][j]; besti = (k * 64 + lane) * 8 + j; }
    // row max, then the lowest column index holding it (DPP lane moves, no LDS)
    const float gmx = wave_max_dpp(mx);
    besti = wave_min_dpp(mx == gmx ? besti : 0x7fffffff);
    mx = gmx;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) s += __expf(z[k][j] - mx);
    s = wave_sum_dpp(s);
    const float lse = mx + __logf(s);
    // the label's logit: the owning lane broadcasts it (the label is row-uniform)
    float zl = 0.f;
    if (valid) {
      const int ok = label >> 3, kk = ok / 64, jj = label & 7;
      const int ln = __builtin_amdgcn_readfirstlane(ok % 64);
      float mine = 0.f;
#pragma unroll
      for (int k = 0; k < NV; ++k)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (k == kk && j == jj) mine = z[k][j];
      zl = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, mine), ln));
    }
    const float loss = valid ? lse - zl : 0.f;
    if (row_loss && lane == 0) row_loss[row] = loss;
    if (valid) { l_sum += loss; n_valid += 1.f; n_correct += (besti == label) ? 1.f : 0.f; }
    if (dlogits) {
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int c0 = (k * 64 + lane) * 8;
        if (c0 < C) {
          unsigned o[4];
#pragma unroll
          for (int j = 0; j < 8; j += 2) {
            float g0 = 0.f, g1 = 0.f;
            if (valid) {
              g0 = (__expf(z[k][j] - lse) - (c0 + j == label ? 1.f : 0.f)) * grad_scale;
              g1 = (__expf(z[k][j + 1] - lse) - (c0 + j + 1 == label ? 1.f : 0.f)) * grad_scale;
            }
            const bf16_t h0 = f2bf(g0), h1 = f2bf(g1);
            o[j >> 1] = (unsigned)h0 | ((unsigned)h1 << 16);
            db[k][j] += bf2f(h0);
            db[k][j + 1] += bf2f(h1);
          }
          u32x4 ov; ov.x = o[0]; ov.y = o[1]; ov.z = o[2]; ov.w = o[3];
          *reinterpret_cast<u32x4*>(dlogits + (long)row * ldd + c0) = ov;
        }
      }
    }
  }
  if (dbias && dlogits) {
#pragma unroll
    for (int k = 0; k < NV; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) part[w][(k * 64 + lane) * 8 + j] = db[k][j];
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256) atomicAdd(dbias + c, part[0][c] + part[1][c] + part[2][c] + part[3][c]);
  }
  // loss, validity and correctness are wave-uniform: lane 0 holds the wave's sums
  if (mslab) {
    // this workgroup's (loss, n, correct) added into its OWN slab row: 4 atomics per
    // workgroup to the same 4 words serialise (6.4 us of an 18.3 us launch at M = 2048,
    // tools/bench_xent.py); adds to distinct rows do not.  Added, not stored: several CE
    // launches (microbatches, possibly on concurrent streams) may land in one step; the
    // step-end fold sums the rows and re-zeroes them (jdt_metrics_fold_slab)
    if (lane == 0) { red[w][0] = l_sum; red[w][1] = n_valid; red[w][2] = n_correct; }
    __syncthreads();
    if (threadIdx.x < 3) {
      const int k = threadIdx.x;
      atomicAdd(reinterpret_cast<float*>(mslab + blockIdx.x) + k, red[0][k] + red[1][k] + red[2][k] + red[3][k]);
    }
  } else if (metrics) {
    xent_metrics_fold(red, w, lane, l_sum, n_valid, n_correct, metrics);
  }
}

}  // namespace jdt
using namespace jdt;

static int g_xent_rpw = 0;
JDT_API void jdt_xent_set_rpw(int r) { g_xent_rpw = r; }  // sweeps: rows per wave of the wide-vocabulary kernel

// mslab (optional, capacity mslab_cap rows of 4 floats, zero on entry): the wide-vocabulary
// kernel stores each workgroup's metric sums in its own row instead of adding them to
// `metrics` (which then is not touched); returns 1 if it did, 0 if `metrics` got them.
JDT_API int jdt_xent_slab(const void* logits, int logits_f32, long ld, const int* labels, int M, int C,
                          float grad_scale, void* dlogits, long ldd, float* dbias, float* metrics, float* row_loss,
                          float* mslab, int mslab_cap, void* stream) {
  if (M <= 0) return 0;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!logits_f32 && C >= 256 && C % 8 == 0 && C <= 2048 && ld % 8 == 0 && ldd % 8 == 0 &&
      (reinterpret_cast<uintptr_t>(logits) & 15) == 0 && (reinterpret_cast<uintptr_t>(dlogits) & 15) == 0) {
    // rows per wave: fewer workgroups = fewer same-address metric atomics, which
    // serialise (tools/bench_xent.py, M = 2048: rpw 4 18.8 us, 2 22.1, 1 32.8;
    // M = 512: rpw 2 10.6, 1 11.5)
    int rpw = M >= 2048 ? 4 : (M >= 512 ? 2 : 1);
    if (g_xent_rpw > 0) rpw = g_xent_rpw;
    dim3 vgrid((M + 4 * rpw - 1) / (4 * rpw));
    float4* slab = (mslab && (int)vgrid.x <= mslab_cap && (reinterpret_cast<uintptr_t>(mslab) & 15) == 0)
                       ? reinterpret_cast<float4*>(mslab) : nullptr;
    auto lg = static_cast<const bf16_t*>(logits);
    auto dl = static_cast<bf16_t*>(dlogits);
    if (C <= 512)
      hipLaunchKernelGGL(xent_vec_kernel<1>, vgrid, dim3(256), 0, st, lg, ld, labels, M, C, rpw, grad_scale, dl, ldd,
                         dbias, metrics, row_loss, slab);
    else if (C <= 1024)
      hipLaunchKernelGGL(xent_vec_kernel<2>, vgrid, dim3(256), 0, st, lg, ld, labels, M, C, rpw, grad_scale, dl, ldd,
                         dbias, metrics, row_loss, slab);
    else
      hipLaunchKernelGGL(xent_vec_kernel<4>, vgrid, dim3(256), 0, st, lg, ld, labels, M, C, rpw, grad_scale, dl, ldd,
                         dbias, metrics, row_loss, slab);
    const int rc = HIP_LAUNCH_CHECK();
    return rc < 0 ? rc : (slab ? 1 : 0);
  }
  dim3 grid((M + 3) / 4);
  if (logits_f32)
    hipLaunchKernelGGL(xent_kernel<true>, grid, dim3(256), 0, st, logits, ld, labels, M, C, grad_scale,
                       static_cast<bf16_t*>(dlogits), ldd, dbias, metrics, row_loss);
  else
    hipLaunchKernelGGL(xent_kernel<false>, grid, dim3(256), 0, st, logits, ld, labels, M, C, grad_scale,
                       static_cast<bf16_t*>(dlogits), ldd, dbias, metrics, row_loss);
  return HIP_LAUNCH_CHECK();
}

JDT_API int jdt_xent(const void* logits, int logits_f32, long ld, const int* labels, int M, int C, float grad_scale,
                     void* dlogits, long ldd, float* dbias, float* metrics, float* row_loss, void* stream) {
  const int rc = jdt_xent_slab(logits, logits_f32, ld, labels, M, C, grad_scale, dlogits, ldd, dbias, metrics, row_loss,
                               nullptr, 0, stream);
  return rc < 0 ? rc : 0;
}
