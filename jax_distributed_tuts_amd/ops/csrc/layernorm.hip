// LayerNorm forward / backward for the transformer tutorial model.
//
// One wave per row (row length d <= 2048, held in registers, 8-element
// 16-byte vector loads per lane); fp32 statistics, bf16 in/out, fp32 affine
// params read from the master buffer.  The backward fuses the residual-branch
// gradient add (dx = dres + LN'(dy)) and reduces dgamma/dbeta per workgroup in
// LDS before one atomic per column per workgroup.
#include "common.h"

namespace jdt {

constexpr int LN_MAXV = 4;  // 4 x 8 x 64 = 2048 columns max

// Row-block index of this workgroup, XCD-contiguous: workgroups are dealt round-robin over
// the 8 XCDs by id, so XCD x takes blocks [x G/8, (x+1) G/8) -- the rows the neighbouring
// GEMMs' tile maps (gemm_dma_kernel: contiguous tile ranges per XCD, row-major) produce and
// consume on that XCD, instead of every 8th block.  JDT_LN_XCD=0 (jdt_ln_set_xcd) restores
// the natural order.
__device__ __forceinline__ int ln_block(int xcd_map) {
  const int G = gridDim.x, b = blockIdx.x;
  if (!xcd_map || (G & 7)) return b;
  return (b & 7) * (G >> 3) + (b >> 3);
}

// Forward: one wave per row.  The affine parameters' loads are issued together
// with the row's (the previous version computed the statistics first and only
// then loaded gamma / beta: a second dependent memory round trip), and the two
// row reductions are DPP lane moves (wave_sum_dpp) instead of ds_bpermute
// butterflies.
//
// EMB: the row is the token + position embedding (the model's first LayerNorm): x =
// wte[tok[row]] + wpe[row % S] (bf16x8_add, the bits embed_fwd_kernel stores) is built in
// registers, stored to E.x (the residual stream) and normalised -- the embedding's own
// launch and its re-read of x go away.
struct LnEmbed {
  const int* tok;
  const bf16_t* wte;
  const bf16_t* wpe;
  int S;
  bf16_t* x;
};

template <int NV, bool EMB>
__global__ void __launch_bounds__(256) ln_fwd_kernel(const bf16_t* __restrict__ x, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, bf16_t* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int T, int d, float eps, int xcd_map, LnEmbed E) {
  const int lane = threadIdx.x & 63;
  const int row = ln_block(xcd_map) * 4 + (threadIdx.x >> 6);
  if (row >= T) return;
  const bf16_t* xr = EMB ? E.wte + (long)E.tok[row] * d : x + (long)row * d;
  const bf16_t* pr = EMB ? E.wpe + (long)(row % E.S) * d : nullptr;
  u32x4 p[NV], pp[NV];
  float4 g[NV][2], bt[NV][2];
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int col = (c * 64 + lane) * 8;
    p[c] = pp[c] = (u32x4){0u, 0u, 0u, 0u};
    g[c][0] = g[c][1] = bt[c][0] = bt[c][1] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (col < d) {
      p[c] = *reinterpret_cast<const u32x4*>(xr + col);
      if (EMB) pp[c] = *reinterpret_cast<const u32x4*>(pr + col);
      g[c][0] = *reinterpret_cast<const float4*>(gamma + col);
      g[c][1] = *reinterpret_cast<const float4*>(gamma + col + 4);
      bt[c][0] = *reinterpret_cast<const float4*>(beta + col);
      bt[c][1] = *reinterpret_cast<const float4*>(beta + col + 4);
    }
  }
  if (EMB) {
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int col = (c * 64 + lane) * 8;
      if (col < d) {
        p[c] = bf16x8_add(p[c], pp[c]);
        *reinterpret_cast<u32x4*>(E.x + (long)row * d + col) = p[c];
      }
    }
  }
  float v[NV][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NV; ++c) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[c][2 * j] = bf2f((bf16_t)(p[c][j] & 0xffff));
      v[c][2 * j + 1] = bf2f((bf16_t)(p[c][j] >> 16));
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[c][j];
  }
  const float mean = __fdiv_rn(wave_sum_dpp(s), (float)d);
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col < d)
#pragma unroll
      for (int j = 0; j < 8; ++j) q = ln_sq_acc(q, v[c][j], mean);
  }
  const float rstd = rsqrtf(__fadd_rn(__fdiv_rn(wave_sum_dpp(q), (float)d), eps));
  if (lane == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int col = (c * 64 + lane) * 8;
    if (col < d) {
      const float gg[8] = {g[c][0].x, g[c][0].y, g[c][0].z, g[c][0].w, g[c][1].x, g[c][1].y, g[c][1].z, g[c][1].w};
      const float bb[8] = {bt[c][0].x, bt[c][0].y, bt[c][0].z, bt[c][0].w,
                           bt[c][1].x, bt[c][1].y, bt[c][1].z, bt[c][1].w};
      u32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float a = ln_norm(v[c][2 * j], mean, rstd, gg[2 * j], bb[2 * j]);
        const float b = ln_norm(v[c][2 * j + 1], mean, rstd, gg[2 * j + 1], bb[2 * j + 1]);
        o[j] = (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16);
      }
      *reinterpret_cast<u32x4*>(y + (long)row * d + col) = o;
    }
  }
}

// Backward: a wave owns R rows whose x / dy / dres loads are all issued before
// any arithmetic; dgamma, dbeta and the optional colsum(dx) are accumulated in
// registers over the wave's rows, summed over the 4 waves in LDS, and added to
// the outputs with one fp32 atomic per column per workgroup.
template <int NV, int R, int W>
__global__ void __launch_bounds__(64 * W) ln_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x,
                                                     const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
                                                     const float* __restrict__ gamma, const bf16_t* __restrict__ dres,
                                                     bf16_t* __restrict__ dx, float* __restrict__ dgamma,
                                                     float* __restrict__ dbeta, float* __restrict__ dsum, int T, int d,
                                                     int xcd_map) {
  __shared__ float part[W][512 * NV];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r0 = (ln_block(xcd_map) * W + w) * R;
  float ag[NV][8], ab[NV][8], ad[NV][8], gm[NV][8];
  u32x4 px[R][NV], pd[R][NV], pr[R][NV];
  float mean[R], rstd[R];
#pragma unroll
  for (int c = 0; c < NV; ++c) {
    const int col = (c * 64 + lane) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) { ag[c][j] = 0.f; ab[c][j] = 0.f; ad[c][j] = 0.f; gm[c][j] = 0.f; }
    if (col < d) {
      const float4 g0 = *reinterpret_cast<const float4*>(gamma + col);
      const float4 g1 = *reinterpret_cast<const float4*>(gamma + col + 4);
      gm[c][0] = g0.x; gm[c][1] = g0.y; gm[c][2] = g0.z; gm[c][3] = g0.w;
      gm[c][4] = g1.x; gm[c][5] = g1.y; gm[c][6] = g1.z; gm[c][7] = g1.w;
    }
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int row = r0 + i;
    const bool ok = row < T;
    mean[i] = ok ? mean_in[row] : 0.f;
    rstd[i] = ok ? rstd_in[row] : 0.f;
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const int col = (c * 64 + lane) * 8;
      const u32x4 zero = {0u, 0u, 0u, 0u};
      px[i][c] = zero; pd[i][c] = zero; pr[i][c] = zero;
      if (ok && col < d) {
        px[i][c] = *reinterpret_cast<const u32x4*>(x + (long)row * d + col);
        pd[i][c] = *reinterpret_cast<const u32x4*>(dy + (long)row * d + col);
        if (dres) pr[i][c] = *reinterpret_cast<const u32x4*>(dres + (long)row * d + col);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int row = r0 + i;
    float xh[NV][8], g[NV][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NV; ++c) {
      const unsigned wx[4] = {px[i][c].x, px[i][c].y, px[i][c].z, px[i][c].w};
      const unsigned wd[4] = {pd[i][c].x, pd[i][c].y, pd[i][c].z, pd[i][c].w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xv = bf2f((bf16_t)((wx[j >> 1] >> (16 * (j & 1))) & 0xffff));
        const float dv = bf2f((bf16_t)((wd[j >> 1] >> (16 * (j & 1))) & 0xffff));
        xh[c][j] = (xv - mean[i]) * rstd[i];
        g[c][j] = dv * gm[c][j];
        s1 += g[c][j];
        s2 += g[c][j] * xh[c][j];
        ag[c][j] += dv * xh[c][j];
        ab[c][j] += dv;
      }
    }
    s1 = wave_sum_dpp(s1) / d;
    s2 = wave_sum_dpp(s2) / d;
    if (row < T) {
#pragma unroll
      for (int c = 0; c < NV; ++c) {
        const int col = (c * 64 + lane) * 8;
        if (col < d) {
          const unsigned wr[4] = {pr[i][c].x, pr[i][c].y, pr[i][c].z, pr[i][c].w};
          unsigned o[4];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float ra = bf2f((bf16_t)(wr[j] & 0xffff)), rb = bf2f((bf16_t)(wr[j] >> 16));
            const float va = ra + rstd[i] * (g[c][2 * j] - s1 - xh[c][2 * j] * s2);
            const float vb = rb + rstd[i] * (g[c][2 * j + 1] - s1 - xh[c][2 * j + 1] * s2);
            const bf16_t ha = f2bf(va), hb = f2bf(vb);
            o[j] = (unsigned)ha | ((unsigned)hb << 16);
            ad[c][2 * j] += bf2f(ha);  // colsum of exactly the stored dx (next layer's bias grad)
            ad[c][2 * j + 1] += bf2f(hb);
          }
          u32x4 ov; ov.x = o[0]; ov.y = o[1]; ov.z = o[2]; ov.w = o[3];
          *reinterpret_cast<u32x4*>(dx + (long)row * d + col) = ov;
        }
      }
    }
  }
  // three column reductions through one LDS image, one atomic per column each
  float (*acc3[3])[8] = {ag, ab, ad};
  float* outs[3] = {dgamma, dbeta, dsum};
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    if (!outs[t]) continue;  // uniform
    __syncthreads();
#pragma unroll
    for (int c = 0; c < NV; ++c)
#pragma unroll
      for (int j = 0; j < 8; ++j) part[w][(c * 64 + lane) * 8 + j] = acc3[t][c][j];
    __syncthreads();
    for (int i = threadIdx.x; i < d; i += 64 * W) {
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < W; ++k) acc += part[k][i];
      atomicAdd(outs[t] + i, acc);
    }
  }
}

}  // namespace jdt
using namespace jdt;

static int g_ln_xcd = 1;
JDT_API void jdt_ln_set_xcd(int on) { g_ln_xcd = on; }

template <bool EMB>
static int ln_fwd_launch(const void* x, const float* gamma, const float* beta, void* y, float* mean, float* rstd, int T,
                         int d, float eps, const LnEmbed& E, void* stream) {
  if (d % 8 || d > 2048) return -3;
  if ((reinterpret_cast<uintptr_t>(gamma) | reinterpret_cast<uintptr_t>(beta) | reinterpret_cast<uintptr_t>(x) |
       reinterpret_cast<uintptr_t>(y)) & 15)
    return -2;
  if (EMB && (E.S <= 0 || ((reinterpret_cast<uintptr_t>(E.wte) | reinterpret_cast<uintptr_t>(E.wpe)) & 15))) return -2;
  const int nv = (d / 8 + 63) / 64;
  dim3 grid((T + 3) / 4);
  hipStream_t st = static_cast<hipStream_t>(stream);
  const bf16_t* xb = static_cast<const bf16_t*>(x);
  bf16_t* yb = static_cast<bf16_t*>(y);
  switch (nv) {
    case 1: hipLaunchKernelGGL((ln_fwd_kernel<1, EMB>), grid, dim3(256), 0, st, xb, gamma, beta, yb, mean, rstd, T, d, eps, g_ln_xcd, E); break;
    case 2: hipLaunchKernelGGL((ln_fwd_kernel<2, EMB>), grid, dim3(256), 0, st, xb, gamma, beta, yb, mean, rstd, T, d, eps, g_ln_xcd, E); break;
    default: hipLaunchKernelGGL((ln_fwd_kernel<4, EMB>), grid, dim3(256), 0, st, xb, gamma, beta, yb, mean, rstd, T, d, eps, g_ln_xcd, E); break;
  }
  return HIP_LAUNCH_CHECK();
}

JDT_API int jdt_ln_fwd(const void* x, const float* gamma, const float* beta, void* y, float* mean, float* rstd, int T,
                       int d, float eps, void* stream) {
  return ln_fwd_launch<false>(x, gamma, beta, y, mean, rstd, T, d, eps, LnEmbed{}, stream);
}

// x_out = wte[tok] + wpe[t % S] (bf16, as jdt_embed_fwd) and y = LN(x_out), one launch
JDT_API int jdt_ln_fwd_embed(const int* tok, const void* wte, const void* wpe, int S, void* x_out, const float* gamma,
                             const float* beta, void* y, float* mean, float* rstd, int T, int d, float eps,
                             void* stream) {
  const LnEmbed E{tok, static_cast<const bf16_t*>(wte), static_cast<const bf16_t*>(wpe), S, static_cast<bf16_t*>(x_out)};
  return ln_fwd_launch<true>(x_out, gamma, beta, y, mean, rstd, T, d, eps, E, stream);
}

static int g_ln_rows = 0, g_ln_waves = 0;
JDT_API void jdt_ln_set_rows(int r) { g_ln_rows = r; }
JDT_API void jdt_ln_set_waves(int w) { g_ln_waves = w; }

// dsum (optional): += colsum(dx), the bias gradient of the layer that produced
// this LayerNorm's input (a residual-stream Dense), so it needs no pass of its own.
JDT_API int jdt_ln_bwd(const void* dy, const void* x, const float* mean, const float* rstd, const float* gamma,
                       const void* dres, void* dx, float* dgamma, float* dbeta, float* dsum, int T, int d,
                       void* stream) {
  if (d % 8 || d > 2048) return -3;
  const int nv = (d / 8 + 63) / 64;
  hipStream_t st = static_cast<hipStream_t>(stream);
  auto a = static_cast<const bf16_t*>(dy);
  auto b = static_cast<const bf16_t*>(x);
  auto r = static_cast<const bf16_t*>(dres);
  auto o = static_cast<bf16_t*>(dx);
  if ((reinterpret_cast<uintptr_t>(gamma) & 15)) return -3;
  // A workgroup = W waves x R rows each.  The column sums cost one same-address
  // atomic per column per workgroup (they serialise in L2), so the rows per
  // workgroup set the atomic count; W spreads those rows over more waves (the
  // per-row work after the loads is serial within a wave).  g_ln_rows /
  // g_ln_waves force R / W (sweeps: tools/bench_ln.py).
  int R = g_ln_rows, W = g_ln_waves;
  if (W == 0) W = (nv <= 2 && T >= 1024) ? 16 : 4;
  if (nv > 2 && W > 4) W = 4;  // LDS image part[W][512 NV]
  if (R == 0) R = W == 16 ? 2 : (T >= 1024 ? 4 : 2);
#define JDT_LNB(NV_, R_, W_)                                                                                      \
  hipLaunchKernelGGL((ln_bwd_kernel<NV_, R_, W_>), dim3((T + W_ * R_ - 1) / (W_ * R_)), dim3(64 * W_), 0, st, a, b, \
                     mean, rstd, gamma, r, o, dgamma, dbeta, dsum, T, d, g_ln_xcd)
  // register budget: R x NV x 3 row vectors per lane -> R <= 2 at 16 waves, <= 4 at 8
  switch (nv) {
    case 1:
      if (W >= 16) { if (R >= 2) JDT_LNB(1, 2, 16); else JDT_LNB(1, 1, 16); }
      else if (W >= 8) { if (R >= 4) JDT_LNB(1, 4, 8); else if (R >= 2) JDT_LNB(1, 2, 8); else JDT_LNB(1, 1, 8); }
      else { if (R >= 8) JDT_LNB(1, 8, 4); else if (R >= 4) JDT_LNB(1, 4, 4); else if (R >= 2) JDT_LNB(1, 2, 4); else JDT_LNB(1, 1, 4); }
      break;
    case 2:
      if (W >= 16) { if (R >= 2) JDT_LNB(2, 2, 16); else JDT_LNB(2, 1, 16); }
      else if (W >= 8) { if (R >= 4) JDT_LNB(2, 4, 8); else if (R >= 2) JDT_LNB(2, 2, 8); else JDT_LNB(2, 1, 8); }
      else { if (R >= 8) JDT_LNB(2, 8, 4); else if (R >= 4) JDT_LNB(2, 4, 4); else if (R >= 2) JDT_LNB(2, 2, 4); else JDT_LNB(2, 1, 4); }
      break;
    default: if (R >= 2) JDT_LNB(4, 2, 4); else JDT_LNB(4, 1, 4); break;
  }
#undef JDT_LNB
  return HIP_LAUNCH_CHECK();
}
