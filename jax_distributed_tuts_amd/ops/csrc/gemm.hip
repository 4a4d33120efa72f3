// Generic bf16 MFMA GEMM for gfx950 with fused epilogues.
//
//   C[M,N] (+)= epilogue( alpha * A[M,K] . B[K,N] )
//
// This one kernel is every dense matmul of the tutorial models (SURVEY K01,
// K05, K09, K11 and the transformer projections):
//   forward   z = x . W + b ; h = dropout(act(z))        (flax Dense, [in,out] kernel)
//   backward  dx = dz . W^T, with the *lower* layer's act'(z) and dropout mask
//             folded into the epilogue (K10) and its bias grad reduced in the
//             epilogue with one atomic per column per wave;
//             dW += x^T . dz accumulated in fp32 in place (beta = 1, K12).
//
// Operands are staged global -> registers -> LDS always in a K-contiguous
// image, so every MFMA fragment read is one 16-byte ds_read.  A source that is
// M/N-contiguous (a transposed operand) is transposed in the register->LDS
// write pass; fp32 sources (input data, fp32 activations) are converted to
// bf16 in the same pass.  Two LDS buffers: the next K-tile's global loads are
// issued before the current tile's MFMAs, written after them (async-stage
// split), one barrier per K-tile.  4 waves per workgroup, each wave owning a
// TM x TN grid of 16x16 fp32 accumulators (v_mfma_f32_16x16x32_bf16).
// Workgroup ids are remapped so neighbouring tiles (which share A rows)
// land on the same XCD's L2.
#include "common.h"

#include <type_traits>

namespace jdt {

struct GemmArgs {
  const void* A; long lda; long sA; int a_f32; int a_trans;  // a_trans: A[m][k] at k*lda+m
  const void* B; long ldb; long sB; int b_f32; int b_trans;  // b_trans=0: B[k][n] at n*ldb+k ; 1: k*ldb+n
  int M, N, K;
  float alpha;
  // forward epilogue
  const void* bias; int bias_f32;          // per-column bias (optional)
  int act;                                  // activation applied after bias
  void* Zout; long ldz; long sZ;            // optional pre-activation store (bf16)
  // backward epilogue: v *= act'(Zin) (Zin bf16, same layout as C)
  const bf16_t* Zin; long ldzin; long sZin; int act_bwd;
  // dropout (forward: applied after act; backward: mask regenerated)
  float keep_prob; unsigned long long seed, offset;
  const void* resid; long ldr; long sR;     // optional residual (bf16) added last
  float* dbias;                             // optional column-sum of the final values (fp32 atomics)
  // output
  void* C; long ldc; long sC; int c_f32; int accumulate;
  // device step counter: dropout offset += step << 32, so a replayed hipGraph
  // draws a fresh mask every step without re-recording kernel arguments
  const int* step_ptr;
  // optional 2-level batch: z -> (z / zin, z % zin) with strides (sX, sX2) for
  // A, B and C (attention: batch x head over the fused [T, 3d] QKV buffer)
  int zin; long sA2, sB2, sC2;
  // optional AdamW in the epilogue of a weight-gradient GEMM whose result is that
  // weight's FINAL gradient of the step (fp32 C only): the element's gradient
  // (C + value if accumulate, else value) updates the fp32 master / m / v views
  // (same layout as C) and the bf16 shadow; C is reset to 0 when it was read.  The
  // step's remaining parameters are updated by adamw_ranges_kernel, which also
  // advances the device step counter (read here as t = step + 1).
  float* opt_p; float* opt_m; float* opt_v; bf16_t* opt_s; const int* opt_step;
  float opt_lr, opt_b1, opt_b2, opt_eps, opt_wd, opt_gs;
  // optional device-resident dropout seed (replaces ``seed``): a hipGraph replayed once
  // per minibatch selects that minibatch's key on the device (util.accum_grads_scan)
  const unsigned long long* seed_ptr;
};

// AdamW of one element in a GEMM epilogue (see GemmArgs::opt_*): optax.adamw, the
// arithmetic of optim.hip adamw_kernel.
struct OptBC { float rbc1, rbc2; };
__device__ __forceinline__ OptBC opt_bc(const GemmArgs& g) {
  OptBC b{1.f, 1.f};
  if (g.opt_p) {
    const int t = g.opt_step[0] + 1;
    b.rbc1 = 1.f / (1.f - powf(g.opt_b1, (float)t));
    b.rbc2 = 1.f / (1.f - powf(g.opt_b2, (float)t));
  }
  return b;
}
__device__ __forceinline__ float opt_update(const GemmArgs& g, const OptBC& bc, long i, float grad) {
  const float gr = grad * g.opt_gs;
  const float mm = g.opt_b1 * g.opt_m[i] + (1.f - g.opt_b1) * gr;
  const float vv = g.opt_b2 * g.opt_v[i] + (1.f - g.opt_b2) * gr * gr;
  float pp = g.opt_p[i];
  pp -= g.opt_lr * ((mm * bc.rbc1) / (sqrtf(vv * bc.rbc2) + g.opt_eps) + g.opt_wd * pp);
  g.opt_m[i] = mm;
  g.opt_v[i] = vv;
  g.opt_p[i] = pp;
  return pp;
}

// Write-through 16-byte store (two relaxed agent-scope 8-byte atomic stores: global_store
// ... sc1): the line goes past this XCD's L2 while the kernel runs instead of staying
// dirty until the kernel-end release writes the L2 back (jdt_gemm_set_wt; A/B).
typedef __attribute__((address_space(1))) unsigned long long gm_u64;
__device__ __forceinline__ void st16(void* p, u32x4 v, bool wt) {
  if (wt) {
    __hip_atomic_store((gm_u64*)p, (unsigned long long)v[0] | ((unsigned long long)v[1] << 32), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store((gm_u64*)p + 1, (unsigned long long)v[2] | ((unsigned long long)v[3] << 32), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  } else {
    *reinterpret_cast<u32x4*>(p) = v;
  }
}
__device__ __forceinline__ void st16f(float* p, float4 x, bool wt) {
  u32x4 v;
  v[0] = __float_as_uint(x.x); v[1] = __float_as_uint(x.y); v[2] = __float_as_uint(x.z); v[3] = __float_as_uint(x.w);
  st16(p, v, wt);
}
// bit 0: C / Zout stores of the vectorised epilogue; bit 1: its AdamW state and shadow stores
__device__ int g_gemm_wt_dev = 0;

// The same for 8 consecutive elements (16-byte aligned): p / m / v as float4 pairs,
// the bf16 shadow as one 16-byte store -- the vectorised epilogue's unit.
__device__ __forceinline__ u32x4 opt_update8(const GemmArgs& g, const OptBC& bc, long i, const float (&grad)[8],
                                             bool wt = false) {
  float4* P4 = reinterpret_cast<float4*>(g.opt_p + i);
  float4* M4 = reinterpret_cast<float4*>(g.opt_m + i);
  float4* V4 = reinterpret_cast<float4*>(g.opt_v + i);
  const float4 p0 = P4[0], p1 = P4[1], m0 = M4[0], m1 = M4[1], v0 = V4[0], v1 = V4[1];
  float p[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
  float m[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
  float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float gr = grad[k] * g.opt_gs;
    m[k] = g.opt_b1 * m[k] + (1.f - g.opt_b1) * gr;
    v[k] = g.opt_b2 * v[k] + (1.f - g.opt_b2) * gr * gr;
    p[k] -= g.opt_lr * ((m[k] * bc.rbc1) / (sqrtf(v[k] * bc.rbc2) + g.opt_eps) + g.opt_wd * p[k]);
  }
  st16f(g.opt_p + i, make_float4(p[0], p[1], p[2], p[3]), wt);
  st16f(g.opt_p + i + 4, make_float4(p[4], p[5], p[6], p[7]), wt);
  st16f(g.opt_m + i, make_float4(m[0], m[1], m[2], m[3]), wt);
  st16f(g.opt_m + i + 4, make_float4(m[4], m[5], m[6], m[7]), wt);
  st16f(g.opt_v + i, make_float4(v[0], v[1], v[2], v[3]), wt);
  st16f(g.opt_v + i + 4, make_float4(v[4], v[5], v[6], v[7]), wt);
  u32x4 o;
#pragma unroll
  for (int k = 0; k < 4; ++k) o[k] = (unsigned)f2bf(p[2 * k]) | ((unsigned)f2bf(p[2 * k + 1]) << 16);
  return o;
}

// opt_update8 with its p / m / v loads issued earlier (gemm_finish_img's prefetch)
struct OptPre { float4 p0, p1, m0, m1, v0, v1; };
__device__ __forceinline__ void opt_load8(const GemmArgs& g, long i, OptPre& o) {
  const float4* P4 = reinterpret_cast<const float4*>(g.opt_p + i);
  const float4* M4 = reinterpret_cast<const float4*>(g.opt_m + i);
  const float4* V4 = reinterpret_cast<const float4*>(g.opt_v + i);
  o.p0 = P4[0]; o.p1 = P4[1]; o.m0 = M4[0]; o.m1 = M4[1]; o.v0 = V4[0]; o.v1 = V4[1];
}
__device__ __forceinline__ u32x4 opt_update8p(const GemmArgs& g, const OptBC& bc, long i, const float (&grad)[8],
                                              const OptPre& o, bool wt) {
  float p[8] = {o.p0.x, o.p0.y, o.p0.z, o.p0.w, o.p1.x, o.p1.y, o.p1.z, o.p1.w};
  float m[8] = {o.m0.x, o.m0.y, o.m0.z, o.m0.w, o.m1.x, o.m1.y, o.m1.z, o.m1.w};
  float v[8] = {o.v0.x, o.v0.y, o.v0.z, o.v0.w, o.v1.x, o.v1.y, o.v1.z, o.v1.w};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float gr = grad[k] * g.opt_gs;
    m[k] = g.opt_b1 * m[k] + (1.f - g.opt_b1) * gr;
    v[k] = g.opt_b2 * v[k] + (1.f - g.opt_b2) * gr * gr;
    p[k] -= g.opt_lr * ((m[k] * bc.rbc1) / (sqrtf(v[k] * bc.rbc2) + g.opt_eps) + g.opt_wd * p[k]);
  }
  st16f(g.opt_p + i, make_float4(p[0], p[1], p[2], p[3]), wt);
  st16f(g.opt_p + i + 4, make_float4(p[4], p[5], p[6], p[7]), wt);
  st16f(g.opt_m + i, make_float4(m[0], m[1], m[2], m[3]), wt);
  st16f(g.opt_m + i + 4, make_float4(m[4], m[5], m[6], m[7]), wt);
  st16f(g.opt_v + i, make_float4(v[0], v[1], v[2], v[3]), wt);
  st16f(g.opt_v + i + 4, make_float4(v[4], v[5], v[6], v[7]), wt);
  u32x4 r;
#pragma unroll
  for (int k = 0; k < 4; ++k) r[k] = (unsigned)f2bf(p[2 * k]) | ((unsigned)f2bf(p[2 * k + 1]) << 16);
  return r;
}

__device__ __forceinline__ long zoff(const GemmArgs& g, int z, long s1, long s2) {
  return g.zin > 1 ? (long)(z / g.zin) * s1 + (long)(z % g.zin) * s2 : (long)z * s1;
}

template <int WM, int WN, int TM, int TN, int BK>
struct Tile {
  static constexpr int BM = WM * TM * 16;
  static constexpr int BN = WN * TN * 16;
  static constexpr int LDK = BK + 8;                  // padded K stride (elements)
  static constexpr int A_CHUNKS = BM * BK / 8;        // 8-element chunks per tile
  static constexpr int B_CHUNKS = BN * BK / 8;
  static constexpr int A_PER_T = (A_CHUNKS + 255) / 256;
  static constexpr int B_PER_T = (B_CHUNKS + 255) / 256;
};

__device__ __forceinline__ unsigned pack2(bf16_t lo, bf16_t hi) { return (unsigned)lo | ((unsigned)hi << 16); }

// Load one 8-element chunk of a (rows x K) operand into packed bf16.
//   non-transposed: elements (r, k0..k0+7) at base + r*ld + k
//   transposed    : elements (r0..r0+7, k) at base + k*ld + r
template <bool F32>
__device__ __forceinline__ u32x4 load_chunk(const void* base, long ld, bool trans, int r, int k,
                                            int R, int K, bool vec_ok) {
  u32x4 out = {0u, 0u, 0u, 0u};
  if (!trans) {
    if (r >= R) return out;
    const long off = (long)r * ld + k;
    if (vec_ok && k + 8 <= K) {
      if (F32) {
        const float4* p = reinterpret_cast<const float4*>(static_cast<const float*>(base) + off);
        const float4 x = p[0], y = p[1];
        out.x = pack2(f2bf(x.x), f2bf(x.y)); out.y = pack2(f2bf(x.z), f2bf(x.w));
        out.z = pack2(f2bf(y.x), f2bf(y.y)); out.w = pack2(f2bf(y.z), f2bf(y.w));
      } else {
        out = *reinterpret_cast<const u32x4*>(static_cast<const bf16_t*>(base) + off);
      }
      return out;
    }
    bf16_t e[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bf16_t v = 0;
      if (k + j < K) v = F32 ? f2bf(static_cast<const float*>(base)[off + j]) : static_cast<const bf16_t*>(base)[off + j];
      e[j] = v;
    }
    out.x = pack2(e[0], e[1]); out.y = pack2(e[2], e[3]); out.z = pack2(e[4], e[5]); out.w = pack2(e[6], e[7]);
    return out;
  } else {
    if (k >= K) return out;
    const long off = (long)k * ld + r;
    if (vec_ok && r + 8 <= R) {
      if (F32) {
        const float4* p = reinterpret_cast<const float4*>(static_cast<const float*>(base) + off);
        const float4 x = p[0], y = p[1];
        out.x = pack2(f2bf(x.x), f2bf(x.y)); out.y = pack2(f2bf(x.z), f2bf(x.w));
        out.z = pack2(f2bf(y.x), f2bf(y.y)); out.w = pack2(f2bf(y.z), f2bf(y.w));
      } else {
        out = *reinterpret_cast<const u32x4*>(static_cast<const bf16_t*>(base) + off);
      }
      return out;
    }
    bf16_t e[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bf16_t v = 0;
      if (r + j < R) v = F32 ? f2bf(static_cast<const float*>(base)[off + j]) : static_cast<const bf16_t*>(base)[off + j];
      e[j] = v;
    }
    out.x = pack2(e[0], e[1]); out.y = pack2(e[2], e[3]); out.z = pack2(e[4], e[5]); out.w = pack2(e[6], e[7]);
    return out;
  }
}

// Raw (unconverted) chunk for the preload path: fp32 sources stay fp32 in
// registers until the LDS write, so no load ever waits on a conversion and
// all K-tiles' loads can be in flight at once.
template <bool F32> struct RawChunk { u32x4 v; };
template <> struct RawChunk<true> { float4 x, y; };

template <bool F32>
__device__ __forceinline__ RawChunk<F32> load_raw(const void* base, long ld, bool trans, int r, int k, int R, int K,
                                                  bool vec_ok) {
  RawChunk<F32> out;
  if constexpr (F32) {
    out.x = make_float4(0.f, 0.f, 0.f, 0.f);
    out.y = out.x;
    const float* src = static_cast<const float*>(base);
    float e[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (!trans) {
      if (r >= R) return out;
      const long off = (long)r * ld + k;
      if (vec_ok && k + 8 <= K) {
        const float4* p = reinterpret_cast<const float4*>(src + off);
        out.x = p[0];
        out.y = p[1];
        return out;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) if (k + j < K) e[j] = src[off + j];
    } else {
      if (k >= K) return out;
      const long off = (long)k * ld + r;
      if (vec_ok && r + 8 <= R) {
        const float4* p = reinterpret_cast<const float4*>(src + off);
        out.x = p[0];
        out.y = p[1];
        return out;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) if (r + j < R) e[j] = src[off + j];
    }
    out.x = make_float4(e[0], e[1], e[2], e[3]);
    out.y = make_float4(e[4], e[5], e[6], e[7]);
  } else {
    out.v = load_chunk<false>(base, ld, trans, r, k, R, K, vec_ok);
  }
  return out;
}

// Interior-tile load: the whole chunk is in bounds and 16-byte aligned, so it is
// one (bf16) or two (fp32) unconditional vector loads.  Keeping guards out of
// this path matters beyond the saved compares: hipcc waits vmcnt(0) at every
// join of a guarded scalar-load fallback, which would serialise the K-tiles.
template <bool F32>
__device__ __forceinline__ RawChunk<F32> load_fast(const void* base, long ld, bool trans, int r, int k) {
  RawChunk<F32> out;
  const long off = trans ? (long)k * ld + r : (long)r * ld + k;
  if constexpr (F32) {
    const float4* p = reinterpret_cast<const float4*>(static_cast<const float*>(base) + off);
    out.x = p[0];
    out.y = p[1];
  } else {
    out.v = *reinterpret_cast<const u32x4*>(static_cast<const bf16_t*>(base) + off);
  }
  return out;
}

template <bool F32>
__device__ __forceinline__ u32x4 raw_to_bf16(const RawChunk<F32>& c) {
  if constexpr (F32) {
    u32x4 o;
    o.x = pack2(f2bf(c.x.x), f2bf(c.x.y)); o.y = pack2(f2bf(c.x.z), f2bf(c.x.w));
    o.z = pack2(f2bf(c.y.x), f2bf(c.y.y)); o.w = pack2(f2bf(c.y.z), f2bf(c.y.w));
    return o;
  } else {
    return c.v;
  }
}

// chunk index c -> (row, k) of the tile for either orientation
template <int BK>
__device__ __forceinline__ int2 chunk_rk(int c, bool trans) {
  return trans ? make_int2((c / BK) * 8, c % BK) : make_int2(c / (BK / 8), (c % (BK / 8)) * 8);
}

template <int LDK>
__device__ __forceinline__ void store_chunk(bf16_t* lds, bool trans, int r, int k, const u32x4& v) {
  if (!trans) {
    *reinterpret_cast<u32x4*>(lds + r * LDK + k) = v;
  } else {
    const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      lds[(r + 2 * j) * LDK + k] = (bf16_t)(w[j] & 0xffffu);
      lds[(r + 2 * j + 1) * LDK + k] = (bf16_t)(w[j] >> 16);
    }
  }
}

// Split-K combine (when splits > 1) + the fused epilogue, shared by every GEMM
// kernel body: `acc` is the wave's TM x TN grid of 16x16 fp32 accumulators of
// the BM x BN tile at (tm0, tn0) of batch z.
template <int BM, int BN, int TM, int TN>
__device__ __forceinline__ void gemm_finish(const GemmArgs& g, f32x4 (&acc)[TM][TN], int tm0, int tn0, int z,
                                            int wid, int wm, int wn, int lane, int tid, int splits, int split,
                                            long tile_id, float* __restrict__ ws, unsigned* counters,
                                            int* lds_flag) {
  // ------------------------------------------------------------- split-K combine
  // Every K-slice writes its fp32 partial tile (slab) with device-scope stores
  // (sc1: written through to the cross-XCD coherence point), waits for them
  // (vmcnt), then draws an arrival ticket; the workgroup that draws the last
  // ticket reads the slabs with device-scope loads and runs the epilogue.  No
  // agent-scope release/acquire fence: on this multi-XCD part those lower to a
  // write-back / invalidate of the whole L2 (buffer_wbl2 / buffer_inv sc1),
  // which cost several us per workgroup; only the slab lines need coherence.
  // The slab layout is the lanes' own accumulator order, so the combine is
  // placement independent.
  if (splits > 1) {
    float* slab0 = ws + tile_id * splits * (BM * BN);
    float* slab = slab0 + (long)split * (BM * BN);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          __hip_atomic_store(slab + (((wid * TM + i) * TN + j) * 64 + lane) * 4 + e, acc[i][j][e], __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = lds_flag;
    if (tid == 0) {
      const unsigned t = __hip_atomic_fetch_add(counters + tile_id, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = (t == (unsigned)(splits - 1));
      if (last) __hip_atomic_store(counters + tile_id, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[i][j][e] = 0.f;
    for (int sp = 0; sp < splits; ++sp) {
      const float* sl = slab0 + (long)sp * (BM * BN);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            acc[i][j][e] += __hip_atomic_load(sl + (((wid * TM + i) * TN + j) * 64 + lane) * 4 + e, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // ------------------------------------------------------------- epilogue
  const bool drop = g.keep_prob < 1.0f;
  const float inv_keep = drop ? 1.0f / g.keep_prob : 1.0f;
  const unsigned long long doff = g.offset + (g.step_ptr ? ((unsigned long long)(unsigned)g.step_ptr[0] << 32) : 0ull);
  const unsigned long long dseed = g.seed_ptr ? g.seed_ptr[0] : g.seed;
  const OptBC obc = opt_bc(g);
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int col = tn0 + (wn * TN + j) * 16 + (lane & 15);
    const bool cok = col < g.N;
    float bval = 0.f;
    if (g.bias && cok) bval = g.bias_f32 ? static_cast<const float*>(g.bias)[col] : bf2f(static_cast<const bf16_t*>(g.bias)[col]);
    float csum = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      // the lane's 4 rows form one dropout group: one Philox call for all 4
      const int row0 = tm0 + (wm * TM + i) * 16 + (lane >> 4) * 4;
      u32x4 dbits = {0u, 0u, 0u, 0u};
      if (drop && cok) dbits = dropout_bits(dseed, doff, dropout_group(z, row0, col, g.M, g.N));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = row0 + e;
        if (cok && row < g.M) {
        float v = g.alpha * acc[i][j][e] + bval;
        if (g.Zout) static_cast<bf16_t*>(g.Zout)[(long)z * g.sZ + (long)row * g.ldz + col] = f2bf(v);
        if (g.Zin) v *= act_grad(g.act_bwd, bf2f(g.Zin[(long)z * g.sZin + (long)row * g.ldzin + col]));
        if (g.act) v = act_fwd(g.act, g.Zout ? round_bf(v) : v);
        if (drop) v = keep_word(dbits, e, g.keep_prob) ? v * inv_keep : 0.f;
        if (g.resid) v += bf2f(static_cast<const bf16_t*>(g.resid)[(long)z * g.sR + (long)row * g.ldr + col]);
        const long co = zoff(g, z, g.sC, g.sC2) + (long)row * g.ldc + col;
        if (g.c_f32 && g.opt_p) {
          float* Cp = static_cast<float*>(g.C) + co;
          g.opt_s[co] = f2bf(opt_update(g, obc, co, g.accumulate ? *Cp + v : v));
          if (g.accumulate) *Cp = 0.f;
        } else if (g.c_f32) {
          float* Cp = static_cast<float*>(g.C) + co;
          *Cp = g.accumulate ? *Cp + v : v;
        } else {
          bf16_t* Cp = static_cast<bf16_t*>(g.C) + co;
          if (g.accumulate) {
            *Cp = f2bf(bf2f(*Cp) + v);
          } else {
            v = round_bf(v);  // the bias grad sums exactly what downstream GEMMs read
            *Cp = f2bf(v);
          }
        }
        csum += v;
        }
      }
    }
    if (g.dbias) {
      csum += __shfl_xor(csum, 16, WAVE);
      csum += __shfl_xor(csum, 32, WAVE);
      if (lane < 16 && cok) atomicAdd(g.dbias + col, csum);
    }
  }
}

// Wide-tile variant (TM * TN >= 16, the 128 x 128 LDS-DMA tiles): the accumulators
// go through an LDS image of the output tile first.  The register epilogue above,
// instantiated with 64 accumulators per lane, is too large for the compiler to
// unroll, and the dynamically indexed accumulator array was then promoted to LDS
// (+64 KB per workgroup, SQ_LDS_BANK_CONFLICT 5.1M per launch) or to scratch.  Here
// the only per-lane indexed loop is the fully unrolled register -> LDS copy; the
// epilogue loop reads the image (one thread per column, one dropout group of 4
// rows per iteration, column-coalesced stores).  Split-K slabs are the image in
// row-major float4 order, combined by the last-arriving slice in slice order.
template <int BM, int BN, int TM, int TN>
__device__ __forceinline__ void gemm_finish_lds(const GemmArgs& g, f32x4 (&acc)[TM][TN], int tm0, int tn0, int z,
                                                int wm, int wn, int lane, int tid, int splits, int split, long tile_id,
                                                float* __restrict__ ws, unsigned* counters, float* img) {
  constexpr int LD = BN + 4;   // padded row (floats)
  static_assert(256 % BN == 0 || BN % 256 == 0, "columns per pass");
  // the caller synchronised: every wave is past its last read of the staging ring
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        img[((wm * TM + i) * 16 + (lane >> 4) * 4 + e) * LD + (wn * TN + j) * 16 + (lane & 15)] = acc[i][j][e];
  __syncthreads();
  if (splits > 1) {
    constexpr int NV = BM * BN / 4;
    float* slab0 = ws + tile_id * splits * (BM * BN);
    float* slab = slab0 + (long)split * (BM * BN);
    for (int v = tid; v < NV; v += 256) {
      const int r = (v * 4) / BN, c = (v * 4) % BN;
      const float4 x = *reinterpret_cast<const float4*>(&img[r * LD + c]);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(sys_u32x4, x),
                                             __builtin_amdgcn_make_buffer_rsrc(slab, (short)0, BM * BN * 4, 0x00020000),
                                             v * 16, 0, 16);  // sc1: written through to the coherence point
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(img + BM * LD);
    if (tid == 0) {
      const unsigned t = __hip_atomic_fetch_add(counters + tile_id, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = (t == (unsigned)(splits - 1));
      if (last) __hip_atomic_store(counters + tile_id, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
    for (int v = tid; v < NV; v += 256) {
      float4 sum = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int sp = 0; sp < splits; ++sp) {
        const sys_u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(
            __builtin_amdgcn_make_buffer_rsrc(slab0 + (long)sp * (BM * BN), (short)0, BM * BN * 4, 0x00020000), v * 16,
            0, 16);  // sc1: past this CU's stale L1
        const float4 x = __builtin_bit_cast(float4, q);
        sum.x += x.x; sum.y += x.y; sum.z += x.z; sum.w += x.w;
      }
      const int r = (v * 4) / BN, c = (v * 4) % BN;
      *reinterpret_cast<float4*>(&img[r * LD + c]) = sum;
    }
    __syncthreads();
  }
  // epilogue: thread -> column c (coalesced), rows in dropout groups of 4
  const bool drop = g.keep_prob < 1.0f;
  const float inv_keep = drop ? 1.0f / g.keep_prob : 1.0f;
  const unsigned long long doff = g.offset + (g.step_ptr ? ((unsigned long long)(unsigned)g.step_ptr[0] << 32) : 0ull);
  const unsigned long long dseed = g.seed_ptr ? g.seed_ptr[0] : g.seed;
  constexpr int CPP = BN < 256 ? BN : 256;      // columns per pass
  constexpr int RGS = 256 / CPP;                 // row groups advanced per pass
  const int cl = tid % CPP;
  const OptBC obc = opt_bc(g);
  for (int cb = 0; cb < BN; cb += CPP) {
    const int col = tn0 + cb + cl;
    const bool cok = col < g.N;
    float bval = 0.f;
    if (g.bias && cok) bval = g.bias_f32 ? static_cast<const float*>(g.bias)[col] : bf2f(static_cast<const bf16_t*>(g.bias)[col]);
    float csum = 0.f;
    for (int rg = tid / CPP; rg < BM / 4; rg += RGS) {
      const int row0 = tm0 + rg * 4;
      u32x4 dbits = {0u, 0u, 0u, 0u};
      if (drop && cok) dbits = dropout_bits(dseed, doff, dropout_group(z, row0, col, g.M, g.N));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = row0 + e;
        if (cok && row < g.M) {
          float v = g.alpha * img[(rg * 4 + e) * LD + cb + cl] + bval;
          if (g.Zout) static_cast<bf16_t*>(g.Zout)[(long)z * g.sZ + (long)row * g.ldz + col] = f2bf(v);
          if (g.Zin) v *= act_grad(g.act_bwd, bf2f(g.Zin[(long)z * g.sZin + (long)row * g.ldzin + col]));
          if (g.act) v = act_fwd(g.act, g.Zout ? round_bf(v) : v);
          if (drop) v = keep_word(dbits, e, g.keep_prob) ? v * inv_keep : 0.f;
          if (g.resid) v += bf2f(static_cast<const bf16_t*>(g.resid)[(long)z * g.sR + (long)row * g.ldr + col]);
          const long co = zoff(g, z, g.sC, g.sC2) + (long)row * g.ldc + col;
          if (g.c_f32 && g.opt_p) {
            float* Cp = static_cast<float*>(g.C) + co;
            g.opt_s[co] = f2bf(opt_update(g, obc, co, g.accumulate ? *Cp + v : v));
            if (g.accumulate) *Cp = 0.f;
          } else if (g.c_f32) {
            float* Cp = static_cast<float*>(g.C) + co;
            *Cp = g.accumulate ? *Cp + v : v;
          } else {
            bf16_t* Cp = static_cast<bf16_t*>(g.C) + co;
            if (g.accumulate) {
              *Cp = f2bf(bf2f(*Cp) + v);
            } else {
              v = round_bf(v);
              *Cp = f2bf(v);
            }
          }
          csum += v;
        }
      }
    }
    if (g.dbias && cok) atomicAdd(g.dbias + col, csum);
  }
}

// Vectorised epilogue (the LDS-DMA kernels whenever every output row is
// 16-byte aligned, see epi_vec_ok): the accumulators go through an LDS image of
// the tile, then each thread owns units of 4 rows x 8 columns -- one dropout
// group per column, 16-byte loads / stores of C, Zout, Zin and resid.  The
// per-element register epilogue above stores 2 bytes per lane in 32-byte row
// pieces; on a 2048 x 2048 output that store pass was ~2x the whole K loop of a
// K = 512 GEMM (tools/gemm_ksweep.py: K = 64 took 13-18 us vs torch's 6).  The
// arithmetic per element is the same sequence as gemm_finish, so results are
// bit-identical.
template <int BM, int BN, int NT = 256>
__device__ __forceinline__ void gemm_finish_img(const GemmArgs& g, int tm0, int tn0, int z, int tid, int splits,
                                                int split, long tile_id, float* __restrict__ ws, unsigned* counters,
                                                float* img);

template <int BM, int BN, int TM, int TN, int NT = 256>
__device__ __forceinline__ void gemm_finish_vec(const GemmArgs& g, f32x4 (&acc)[TM][TN], int tm0, int tn0, int z,
                                                int wm, int wn, int lane, int tid, int splits, int split, long tile_id,
                                                float* __restrict__ ws, unsigned* counters, float* img) {
  constexpr int LD = BN + 4;      // padded image row (floats)
  // the caller synchronised: every wave is past its last read of the staging ring
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        img[((wm * TM + i) * 16 + (lane >> 4) * 4 + e) * LD + (wn * TN + j) * 16 + (lane & 15)] = acc[i][j][e];
  gemm_finish_img<BM, BN, NT>(g, tm0, tn0, z, tid, splits, split, tile_id, ws, counters, img);
}

// The same for a wave's TM x TN grid of 32x32 accumulators (v_mfma_f32_32x32x16_bf16:
// lane l holds column l & 31, rows (e & 3) + 8 (e >> 2) + 4 (l >> 5) of register e).
template <int BM, int BN, int TM, int TN, int NT = 256>
__device__ __forceinline__ void gemm_finish_vec32(const GemmArgs& g, f32x16 (&acc)[TM][TN], int tm0, int tn0, int z,
                                                  int wm, int wn, int lane, int tid, int splits, int split,
                                                  long tile_id, float* __restrict__ ws, unsigned* counters,
                                                  float* img) {
  constexpr int LD = BN + 4;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e)
        img[((wm * TM + i) * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5)) * LD + (wn * TN + j) * 32 + (lane & 31)] =
            acc[i][j][e];
  gemm_finish_img<BM, BN, NT>(g, tm0, tn0, z, tid, splits, split, tile_id, ws, counters, img);
}

// Split-K combine + fused epilogue from the fp32 tile image ``img`` ([BM][BN + 4]).
template <int BM, int BN, int NT>
__device__ __forceinline__ void gemm_finish_img(const GemmArgs& g, int tm0, int tn0, int z, int tid, int splits,
                                                int split, long tile_id, float* __restrict__ ws, unsigned* counters,
                                                float* img) {
  constexpr int LD = BN + 4;      // padded image row (floats)
  constexpr int CU = BN / 8;      // 8-column chunks per row
  constexpr int NU = BM / 4 * CU; // 4 x 8 units per tile
  static_assert(NT % CU == 0, "a thread keeps its column chunk across units");
  __syncthreads();
  if (splits > 1) {
    constexpr int NV = BM * BN / 4;
    float* slab0 = ws + tile_id * splits * (BM * BN);
    float* slab = slab0 + (long)split * (BM * BN);
    for (int v = tid; v < NV; v += NT) {
      const int r = (v * 4) / BN, c = (v * 4) % BN;
      const float4 x = *reinterpret_cast<const float4*>(&img[r * LD + c]);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(sys_u32x4, x),
                                             __builtin_amdgcn_make_buffer_rsrc(slab, (short)0, BM * BN * 4, 0x00020000),
                                             v * 16, 0, 16);  // sc1: written through to the coherence point
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(img + BM * LD);
    if (tid == 0) {
      const unsigned t = __hip_atomic_fetch_add(counters + tile_id, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = (t == (unsigned)(splits - 1));
      if (last) __hip_atomic_store(counters + tile_id, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
    for (int v = tid; v < NV; v += NT) {
      float4 sum = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int sp = 0; sp < splits; ++sp) {
        const sys_u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(
            __builtin_amdgcn_make_buffer_rsrc(slab0 + (long)sp * (BM * BN), (short)0, BM * BN * 4, 0x00020000), v * 16,
            0, 16);  // sc1: past this CU's stale L1
        const float4 x = __builtin_bit_cast(float4, q);
        sum.x += x.x; sum.y += x.y; sum.z += x.z; sum.w += x.w;
      }
      const int r = (v * 4) / BN, c = (v * 4) % BN;
      *reinterpret_cast<float4*>(&img[r * LD + c]) = sum;
    }
    __syncthreads();
  }
  const bool drop = g.keep_prob < 1.0f;
  const float inv_keep = drop ? 1.0f / g.keep_prob : 1.0f;
  const unsigned long long doff = g.offset + (g.step_ptr ? ((unsigned long long)(unsigned)g.step_ptr[0] << 32) : 0ull);
  const unsigned long long dseed = g.seed_ptr ? g.seed_ptr[0] : g.seed;
  const int cc = tid % CU;
  const int col = tn0 + cc * 8;
  float bv[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) bv[k] = 0.f;
  if (g.bias) {
    if (g.bias_f32) {
      const float4 b0 = *reinterpret_cast<const float4*>(static_cast<const float*>(g.bias) + col);
      const float4 b1 = *reinterpret_cast<const float4*>(static_cast<const float*>(g.bias) + col + 4);
      bv[0] = b0.x; bv[1] = b0.y; bv[2] = b0.z; bv[3] = b0.w; bv[4] = b1.x; bv[5] = b1.y; bv[6] = b1.z; bv[7] = b1.w;
    } else {
      const u32x4 p = *reinterpret_cast<const u32x4*>(static_cast<const bf16_t*>(g.bias) + col);
#pragma unroll
      for (int k = 0; k < 8; ++k) bv[k] = bf2f((bf16_t)((p[k >> 1] >> (16 * (k & 1))) & 0xffff));
    }
  }
  float cs[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) cs[k] = 0.f;
  const long cbase = zoff(g, z, g.sC, g.sC2);
  const OptBC obc = opt_bc(g);
  const int wtm = g_gemm_wt_dev;
  const bool wt_c = wtm & 1, wt_o = (wtm >> 1) & 1;
  // rows per unit: one dropout group (4 rows) with dropout, else ONE row -- on a 32-row
  // tile that is 4x the threads of the epilogue busy (NU = one wave's worth of 4-row
  // units), which matters for the memory-heavy epilogues (fused AdamW: 26 B/element)
  const int RU = drop ? 4 : 1;
  const int nu = NU * (4 / RU);
  // one unit; pre: its Zin / resid / AdamW-state loads were issued up front (zp, rp, op)
  auto unit = [&](int u, bool pre, u32x4 zp, u32x4 rp, const OptPre& op) __attribute__((always_inline)) {
    const int rl = (u / CU) * RU;  // first row of the unit within the tile
    const int row0 = tm0 + rl;
    u32x4 db[8];
    if (drop) {
#pragma unroll
      for (int k = 0; k < 8; ++k) db[k] = dropout_bits(dseed, doff, dropout_group(z, row0, col + k, g.M, g.N));
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (e >= RU) break;
      const int row = row0 + e;
      float v[8];
      {
        const float4 x0 = *reinterpret_cast<const float4*>(&img[(rl + e) * LD + cc * 8]);
        const float4 x1 = *reinterpret_cast<const float4*>(&img[(rl + e) * LD + cc * 8 + 4]);
        v[0] = x0.x; v[1] = x0.y; v[2] = x0.z; v[3] = x0.w; v[4] = x1.x; v[5] = x1.y; v[6] = x1.z; v[7] = x1.w;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = g.alpha * v[k] + bv[k];
      if (g.Zout) {
        u32x4 o;
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = (unsigned)f2bf(v[2 * k]) | ((unsigned)f2bf(v[2 * k + 1]) << 16);
        st16(static_cast<bf16_t*>(g.Zout) + (long)z * g.sZ + (long)row * g.ldz + col, o, wt_c);
      }
      if (g.Zin) {
        const u32x4 p = pre ? zp : *reinterpret_cast<const u32x4*>(g.Zin + (long)z * g.sZin + (long)row * g.ldzin + col);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] *= act_grad(g.act_bwd, bf2f((bf16_t)((p[k >> 1] >> (16 * (k & 1))) & 0xffff)));
      }
      if (g.act) {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = act_fwd(g.act, g.Zout ? round_bf(v[k]) : v[k]);
      }
      if (drop) {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = keep_word(db[k], e, g.keep_prob) ? v[k] * inv_keep : 0.f;
      }
      if (g.resid) {
        const u32x4 p = pre ? rp : *reinterpret_cast<const u32x4*>(static_cast<const bf16_t*>(g.resid) + (long)z * g.sR +
                                                                    (long)row * g.ldr + col);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] += bf2f((bf16_t)((p[k >> 1] >> (16 * (k & 1))) & 0xffff));
      }
      const long co = cbase + (long)row * g.ldc + col;
      if (g.c_f32 && g.opt_p) {
        float4* Cp = reinterpret_cast<float4*>(static_cast<float*>(g.C) + co);
        if (g.accumulate) {
          const float4 c0 = Cp[0], c1 = Cp[1];
          v[0] += c0.x; v[1] += c0.y; v[2] += c0.z; v[3] += c0.w;
          v[4] += c1.x; v[5] += c1.y; v[6] += c1.z; v[7] += c1.w;
          Cp[0] = make_float4(0.f, 0.f, 0.f, 0.f);
          Cp[1] = Cp[0];
        }
        st16(g.opt_s + co, pre ? opt_update8p(g, obc, co, v, op, wt_o) : opt_update8(g, obc, co, v, wt_o), wt_o);
      } else if (g.c_f32) {
        float4* Cp = reinterpret_cast<float4*>(static_cast<float*>(g.C) + co);
        float4 o0 = make_float4(v[0], v[1], v[2], v[3]), o1 = make_float4(v[4], v[5], v[6], v[7]);
        if (g.accumulate) {
          const float4 c0 = Cp[0], c1 = Cp[1];
          o0.x = c0.x + o0.x; o0.y = c0.y + o0.y; o0.z = c0.z + o0.z; o0.w = c0.w + o0.w;
          o1.x = c1.x + o1.x; o1.y = c1.y + o1.y; o1.z = c1.z + o1.z; o1.w = c1.w + o1.w;
        }
        st16f(reinterpret_cast<float*>(Cp), o0, wt_c);
        st16f(reinterpret_cast<float*>(Cp + 1), o1, wt_c);
      } else {
        u32x4* Cp = reinterpret_cast<u32x4*>(static_cast<bf16_t*>(g.C) + co);
        u32x4 o;
        if (g.accumulate) {
          const u32x4 p = *Cp;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float a = bf2f((bf16_t)(p[k] & 0xffff)) + v[2 * k];
            const float b = bf2f((bf16_t)(p[k] >> 16)) + v[2 * k + 1];
            o[k] = (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16);
          }
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] = round_bf(v[k]);  // the bias grad sums exactly what is stored
#pragma unroll
          for (int k = 0; k < 4; ++k) o[k] = (unsigned)f2bf(v[2 * k]) | ((unsigned)f2bf(v[2 * k + 1]) << 16);
        }
        st16(Cp, o, wt_c);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) cs[k] += v[k];
    }
  };
  if (!drop) {
    // single-row units: every unit's global loads first, then the units -- one memory
    // round trip per thread instead of one per unit (the loads would otherwise wait
    // behind the previous unit's stores, which may alias them; 4 units per thread on a
    // 128 x 128 tile: the GELU' epilogue of the LM's fc2 dX cost 6.5 us over its main loop)
    constexpr int UPT = (BM * CU + NT - 1) / NT;
    constexpr int PB = UPT < 2 ? UPT : 2;   // units prefetched at once (AdamW state: 24 VGPRs each)
#pragma unroll
    for (int b0 = 0; b0 < UPT; b0 += PB) {
      u32x4 zpf[PB], rpf[PB];
      OptPre opf[PB];
#pragma unroll
      for (int j = 0; j < PB; ++j) {
        const int u = tid + (b0 + j) * NT;
        if (u < nu) {
          const int row = tm0 + u / CU;
          if (g.Zin) zpf[j] = *reinterpret_cast<const u32x4*>(g.Zin + (long)z * g.sZin + (long)row * g.ldzin + col);
          if (g.resid)
            rpf[j] = *reinterpret_cast<const u32x4*>(static_cast<const bf16_t*>(g.resid) + (long)z * g.sR +
                                                     (long)row * g.ldr + col);
          if (g.c_f32 && g.opt_p) opt_load8(g, cbase + (long)row * g.ldc + col, opf[j]);
        }
      }
#pragma unroll
      for (int j = 0; j < PB; ++j) {
        const int u = tid + (b0 + j) * NT;
        if (u < nu) unit(u, true, zpf[j], rpf[j], opf[j]);
      }
    }
  } else {
    const OptPre none{};
    for (int u = tid; u < nu; u += NT) unit(u, false, u32x4{0u, 0u, 0u, 0u}, u32x4{0u, 0u, 0u, 0u}, none);
  }
  if (g.dbias) {
    // column sums: the threads sharing a chunk (tid % CU) meet in the image
    constexpr int RPT = NT / CU;  // threads per chunk
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) img[(tid / CU) * (BN + 1) + cc * 8 + k] = cs[k];
    __syncthreads();
    for (int c = tid; c < BN; c += NT) {
      float s = 0.f;
      for (int r = 0; r < RPT; ++r) s += img[r * (BN + 1) + c];
      atomicAdd(g.dbias + tn0 + c, s);
    }
  }
}

// Host: gemm_finish_vec's 16-byte accesses need every row of C / Zout / Zin /
// resid (and every batch / sub-batch slice) to start 16-byte aligned.
static bool epi_vec_ok(const GemmArgs& g, int batch) {
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  auto rows = [&](const void* p, long ld, long s1, long s2, int f32) {
    if (!p) return true;
    const long q = f32 ? 4 : 8;
    return al(p) && ld % q == 0 && (batch <= 1 || (s1 % q == 0 && (g.zin <= 1 || s2 % q == 0)));
  };
  return rows(g.C, g.ldc, g.sC, g.sC2, g.c_f32) && rows(g.Zout, g.ldz, g.sZ, 0, 0) && rows(g.Zin, g.ldzin, g.sZin, 0, 0) &&
         rows(g.resid, g.ldr, g.sR, 0, 0) && (!g.bias || al(g.bias)) && g.N % 8 == 0 &&
         (!g.opt_s || (al(g.opt_s) && al(g.opt_p) && al(g.opt_m) && al(g.opt_v) && g.ldc % 8 == 0));  // fused AdamW: 16-byte accesses
}

template <int WM, int WN, int TM, int TN, int BK, bool AF32, bool BF32, int PRE, bool EXACT = false>
__global__ void __launch_bounds__(256) gemm_kernel(GemmArgs g, int tiles_n, int vecA, int vecB, int splits,
                                                   int kchunk, float* __restrict__ ws, unsigned* counters, int vec) {
  using T = Tile<WM, WN, TM, TN, BK>;
  constexpr int BM = T::BM, BN = T::BN, LDK = T::LDK;
  // EXACT slices keep the whole K-slice resident (one image, one barrier);
  // the other paths double-buffer one K-tile.
  constexpr int LDX = PRE * BK + 8;
  constexpr int SMEM = EXACT ? (BM + BN) * LDX : 2 * (BM + BN) * LDK;
  __shared__ __attribute__((aligned(16))) bf16_t smem[SMEM];
  // buffer b: A image at smem + b*(BM+BN)*LDK, B image right after it
#define AS(b) (smem + (b) * (BM + BN) * LDK)
#define BS(b) (smem + (b) * (BM + BN) * LDK + BM * LDK)

  // XCD-aware bijective remap: blocks b, b+8, ... share an XCD; give each XCD
  // a contiguous run of tiles (cdna_hip_programming.md §5, T1).
  const int nwg = gridDim.x;
  int bid = blockIdx.x;
  {
    const int xcd = bid % 8, q = nwg / 8, rr = nwg % 8;
    bid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
  }
  const int tm0 = (bid / tiles_n) * BM;
  const int tn0 = (bid % tiles_n) * BN;
  const int z = blockIdx.z;

  const void* Ab = static_cast<const char*>(g.A) + zoff(g, z, g.sA, g.sA2) * (AF32 ? 4 : 2);
  const void* Bb = static_cast<const char*>(g.B) + zoff(g, z, g.sB, g.sB2) * (BF32 ? 4 : 2);
  // shift operand bases to this tile
  const long a_off = g.a_trans ? (long)tm0 : (long)tm0 * g.lda;
  const long b_off = g.b_trans ? (long)tn0 : (long)tn0 * g.ldb;
  Ab = static_cast<const char*>(Ab) + a_off * (AF32 ? 4 : 2);
  Bb = static_cast<const char*>(Bb) + b_off * (BF32 ? 4 : 2);
  const int Ar = g.M - tm0, Br = g.N - tn0;  // remaining rows of each operand

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  u32x4 ra[T::A_PER_T], rb[T::B_PER_T];
  // split-K: this workgroup reduces K range [kbeg, kend)
  const int split = blockIdx.y;
  const int kbeg = split * kchunk;
  const int kend = min(g.K, kbeg + kchunk);
  const int nkt = (kend - kbeg + BK - 1) / BK;

  auto gload = [&](int kt) {
    const int kb = kbeg + kt * BK;
#pragma unroll
    for (int i = 0; i < T::A_PER_T; ++i) {
      const int c = tid + i * 256;
      if (c < T::A_CHUNKS) {
        const int2 rk = chunk_rk<BK>(c, g.a_trans); const int r = rk.x, k = rk.y;
        ra[i] = load_chunk<AF32>(Ab, g.lda, g.a_trans, r, kb + k, Ar, kend, vecA);
      }
    }
#pragma unroll
    for (int i = 0; i < T::B_PER_T; ++i) {
      const int c = tid + i * 256;
      if (c < T::B_CHUNKS) {
        const int2 rk = chunk_rk<BK>(c, g.b_trans); const int r = rk.x, k = rk.y;
        rb[i] = load_chunk<BF32>(Bb, g.ldb, g.b_trans, r, kb + k, Br, kend, vecB);
      }
    }
  };
  auto lwrite = [&](int buf) {
#pragma unroll
    for (int i = 0; i < T::A_PER_T; ++i) {
      const int c = tid + i * 256;
      if (c < T::A_CHUNKS) { const int2 rk = chunk_rk<BK>(c, g.a_trans); const int r = rk.x, k = rk.y; store_chunk<LDK>(AS(buf), g.a_trans, r, k, ra[i]); }
    }
#pragma unroll
    for (int i = 0; i < T::B_PER_T; ++i) {
      const int c = tid + i * 256;
      if (c < T::B_CHUNKS) { const int2 rk = chunk_rk<BK>(c, g.b_trans); const int r = rk.x, k = rk.y; store_chunk<LDK>(BS(buf), g.b_trans, r, k, rb[i]); }
    }
  };

  auto mfma_tile = [&](int cur) {
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = (wm * TM + i) * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8*>(AS(cur) + row * LDK + kk + 8 * (lane >> 4));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = (wn * TN + j) * 16 + (lane & 15);
        bfr[j] = *reinterpret_cast<const bf16x8*>(BS(cur) + col * LDK + kk + 8 * (lane >> 4));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(af[i], bfr[j], acc[i][j]);
    }
  };

  if constexpr (EXACT) {
    // Exact slice (host-checked: every tile interior, aligned rows, and this
    // slice is exactly PRE K-tiles): straight-line code with no runtime guard,
    // so hipcc issues all PRE K-tiles' loads back to back and retires them with
    // counted vmcnt waits while they are written into ONE LDS image of the
    // whole slice -- one global round trip, one barrier, then every MFMA of the
    // slice back to back (no per-K-tile barrier: at these sizes the barrier
    // chain, not the MFMA, was the cost).
    bf16_t* As = smem;
    bf16_t* Bs = smem + BM * LDX;
    RawChunk<AF32> pa[PRE][T::A_PER_T];
    RawChunk<BF32> pb[PRE][T::B_PER_T];
#pragma unroll
    for (int kt = 0; kt < PRE; ++kt) {
      const int kb = kbeg + kt * BK;
#pragma unroll
      for (int i = 0; i < T::A_PER_T; ++i) {
        const int c = tid + i * 256;
        if (T::A_CHUNKS % 256 == 0 || c < T::A_CHUNKS) {
          const int2 rk = chunk_rk<BK>(c, g.a_trans);
          pa[kt][i] = load_fast<AF32>(Ab, g.lda, g.a_trans, rk.x, kb + rk.y);
        }
      }
#pragma unroll
      for (int i = 0; i < T::B_PER_T; ++i) {
        const int c = tid + i * 256;
        if (T::B_CHUNKS % 256 == 0 || c < T::B_CHUNKS) {
          const int2 rk = chunk_rk<BK>(c, g.b_trans);
          pb[kt][i] = load_fast<BF32>(Bb, g.ldb, g.b_trans, rk.x, kb + rk.y);
        }
      }
      // keep the issue order = consumption order, so the waits are counted
      // (vmcnt(N)) instead of the scheduler putting tile 0's loads last
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int kt = 0; kt < PRE; ++kt) {
#pragma unroll
      for (int i = 0; i < T::A_PER_T; ++i) {
        const int c = tid + i * 256;
        if (T::A_CHUNKS % 256 == 0 || c < T::A_CHUNKS) {
          const int2 rk = chunk_rk<BK>(c, g.a_trans);
          store_chunk<LDX>(As, g.a_trans, rk.x, kt * BK + rk.y, raw_to_bf16<AF32>(pa[kt][i]));
        }
      }
#pragma unroll
      for (int i = 0; i < T::B_PER_T; ++i) {
        const int c = tid + i * 256;
        if (T::B_CHUNKS % 256 == 0 || c < T::B_CHUNKS) {
          const int2 rk = chunk_rk<BK>(c, g.b_trans);
          store_chunk<LDX>(Bs, g.b_trans, rk.x, kt * BK + rk.y, raw_to_bf16<BF32>(pb[kt][i]));
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < PRE * BK; kk += 32) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = (wm * TM + i) * 16 + (lane & 15);
        af[i] = *reinterpret_cast<const bf16x8*>(As + row * LDX + kk + 8 * (lane >> 4));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = (wn * TN + j) * 16 + (lane & 15);
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + col * LDX + kk + 8 * (lane >> 4));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(af[i], bfr[j], acc[i][j]);
    }
  } else if constexpr (PRE > 0) {
    // Preload: every K-tile of this slice is requested before the first MFMA
    // (nkt <= PRE), so the slice costs ONE global round trip instead of nkt
    // dependent ones; the tiles then stream through the two LDS buffers.
    RawChunk<AF32> pa[PRE][T::A_PER_T];
    RawChunk<BF32> pb[PRE][T::B_PER_T];
#pragma unroll
    for (int kt = 0; kt < PRE; ++kt) {
      if (kt < nkt) {
        const int kb = kbeg + kt * BK;
#pragma unroll
        for (int i = 0; i < T::A_PER_T; ++i) {
          const int c = tid + i * 256;
          if (c < T::A_CHUNKS) {
            const int2 rk = chunk_rk<BK>(c, g.a_trans);
            pa[kt][i] = load_raw<AF32>(Ab, g.lda, g.a_trans, rk.x, kb + rk.y, Ar, kend, vecA);
          }
        }
#pragma unroll
        for (int i = 0; i < T::B_PER_T; ++i) {
          const int c = tid + i * 256;
          if (c < T::B_CHUNKS) {
            const int2 rk = chunk_rk<BK>(c, g.b_trans);
            pb[kt][i] = load_raw<BF32>(Bb, g.ldb, g.b_trans, rk.x, kb + rk.y, Br, kend, vecB);
          }
        }
      }
    }
#pragma unroll
    for (int kt = 0; kt < PRE; ++kt) {
      if (kt < nkt) {
        const int cur = kt & 1;
#pragma unroll
        for (int i = 0; i < T::A_PER_T; ++i) {
          const int c = tid + i * 256;
          if (c < T::A_CHUNKS) {
            const int2 rk = chunk_rk<BK>(c, g.a_trans);
            store_chunk<LDK>(AS(cur), g.a_trans, rk.x, rk.y, raw_to_bf16<AF32>(pa[kt][i]));
          }
        }
#pragma unroll
        for (int i = 0; i < T::B_PER_T; ++i) {
          const int c = tid + i * 256;
          if (c < T::B_CHUNKS) {
            const int2 rk = chunk_rk<BK>(c, g.b_trans);
            store_chunk<LDK>(BS(cur), g.b_trans, rk.x, rk.y, raw_to_bf16<BF32>(pb[kt][i]));
          }
        }
        __syncthreads();
        mfma_tile(cur);
      }
    }
  } else {
    gload(0);
    lwrite(0);
    __syncthreads();
    for (int kt = 0; kt < nkt; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nkt) gload(kt + 1);  // in flight under the MFMAs below
      mfma_tile(cur);
      if (kt + 1 < nkt) lwrite(cur ^ 1);
      __syncthreads();
    }
  }

#undef AS
#undef BS

  if constexpr (BM * BN >= 2048 && (BM * (BN + 4) + 4) * 4 <= SMEM * 2) {
    // interior tiles of a 16-byte-aligned output: the vectorised LDS-image epilogue
    if (vec && tm0 + BM <= g.M && tn0 + BN <= g.N) {
      __syncthreads();  // every wave is past its last read of the staging images
      gemm_finish_vec<BM, BN, TM, TN>(g, acc, tm0, tn0, z, wm, wn, lane, tid, splits, split,
                                      (long)z * gridDim.x + bid, ws, counters, reinterpret_cast<float*>(smem));
      return;
    }
  }
  gemm_finish<BM, BN, TM, TN>(g, acc, tm0, tn0, z, wid, wm, wn, lane, tid, splits, split, (long)z * gridDim.x + bid,
                              ws, counters, reinterpret_cast<int*>(smem));
}


// ---------------------------------------------------------------------------
// LDS-DMA GEMM body (bf16 operands, every tile interior, K-slices a whole
// number of 64-deep K-tiles).  Operand tiles go global -> LDS with
// global_load_lds_dwordx4 (no VGPR staging, no ds_write), S-deep ring of LDS
// stages with ONE barrier per K-tile and a counted vmcnt that keeps the next
// stage in flight across it (cdna_hip_programming.md §5 "Pipelining across
// barriers").  Either operand may be K-contiguous ("mk" A / "nk" B: row image,
// 16-byte chunks XOR-swizzled by row so the ds_read_b128 fragment reads spread
// over the banks) or M/N-contiguous ("km" A / "kn" B, e.g. the [in,out] weight
// of a forward pass or the token-major operands of a weight gradient: k-row
// image read with the gfx950 transposing ds_read_b64_tr_b16, so no operand is
// ever transposed in memory).
constexpr int DMA_BK = 64;

// k-row image swizzle: 16-byte chunk c of k-row r is stored at chunk c ^ tr_swz(r).
// A transposed fragment read has each 32-lane half touch k-rows {0..3, 8..11}
// (+ kk) over the same 16 columns; the XOR puts those 8 rows' 32-byte pieces in
// 8 distinct bank groups (PMC: SQ_LDS_BANK_CONFLICT of the both-transposed
// weight-gradient GEMM 524k -> see profiles).  Rows r and r + 4 share a mask, so
// the second read of a fragment is still the first one's address + 4 rows.
template <int EXT>
__device__ __forceinline__ int tr_swz(int r) {
  if constexpr (EXT == 32) return ((r >> 3) & 1) << 1;
  else if constexpr (EXT == 64) return (((r >> 1) & 1) | (((r >> 3) & 1) << 1)) << 1;
  else return ((r & 3) | (((r >> 3) & 1) << 2)) << 1;  // 128
}

template <int EXT>  // EXT = extent of the non-K dim of the tile (BM or BN)
__device__ __forceinline__ bf16x8 dma_frag(const bf16_t* img, bool kmajor_img, int base, int kk, int lane) {
  if (!kmajor_img) {
    // row image [EXT][64]: row r, 16-byte chunk c lives at slot c ^ (r & 7)
    const int r = base + (lane & 15);
    const int c = (kk >> 3) + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(img + r * DMA_BK + ((c ^ (r & 7)) << 3));
  }
  // k-row image [64][EXT]: lane 4q+p of each 16-lane group addresses k-row q,
  // columns 4p..4p+3 of the group's 4-row block; it receives column (lane & 15).
  // Issued as inline asm: hipcc treats the ds_read_tr intrinsic as aliasing the
  // in-flight LDS-DMA and would wait vmcnt(0) before it, draining the ring.
  // The caller waits lgkmcnt(0) before the MFMAs read the fragments.
  typedef __attribute__((ext_vector_type(4))) short s4;
  const int i16 = lane & 15, k1 = kk + 8 * (lane >> 4) + (i16 >> 2);
  const int col = base + 4 * (i16 & 3);
  const int pcol = (((col >> 3) ^ tr_swz<EXT>(k1)) << 3) | (col & 7);
  const unsigned a0 = (unsigned)(uintptr_t)((__attribute__((address_space(3))) const bf16_t*)(img + k1 * EXT + pcol));
  s4 lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(a0));
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(a0), "n"(4 * EXT * 2));
  bf16x8 f;
  f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
  f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
  return f;
}

// Stage one operand tile (EXT x 64 of a K-contiguous source, or 64 x EXT of an
// EXT-contiguous one) into its LDS image: EXT/32 wave-instructions per wave.
template <int EXT, bool KMAJ, int NW = 4>
__device__ __forceinline__ void dma_stage(const bf16_t* src, long ld, int k0, bf16_t* img, int wid, int lane) {
  constexpr int IPW = EXT / (8 * NW);  // 1 KiB per wave-instruction, EXT*64*2 bytes per tile, NW waves
  static_assert(IPW >= 1, "every wave issues at least one piece");
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int ins = wid * IPW + i;
    const int p = ins * 64 + lane;  // 16-byte slot of the image
    const bf16_t* gp;
    if (!KMAJ) {
      const int r = p >> 3, c = (p & 7) ^ (r & 7);
      gp = src + (long)r * ld + k0 + c * 8;
    } else {
      constexpr int CPR = EXT / 8;  // chunks per k-row
      const int kr = p / CPR, cm = (p % CPR) ^ tr_swz<EXT>(kr);
      gp = src + (long)(k0 + kr) * ld + cm * 8;
    }
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gp,
                                     (__attribute__((address_space(3))) void*)(img + ins * 512), 16, 0, 0);
  }
}

// Tiles wider than 64 on an EXT-contiguous (k-row image) operand are staged as
// EXT/64 side-by-side [64][64] images: a 128-wide k-row is one whole 256-byte LDS
// bank row, so its transposed fragment reads conflicted (PMC on 128 x 128 tiles:
// SQ_LDS_BANK_CONFLICT 5.1M cycles per launch, 2.6x the kernel time of 64 x 64
// tiles); 64-wide sub-images keep the conflict-free EXT = 64 swizzle.
template <int EXT, bool KMAJ, int NW = 4>
__device__ __forceinline__ void stage_op(const bf16_t* src, long ld, int k0, bf16_t* img, int wid, int lane) {
  if constexpr (KMAJ && EXT > 64) {
#pragma unroll
    for (int h = 0; h < EXT / 64; ++h)
      dma_stage<64, true, NW>(src + h * 64, ld, k0, img + h * 64 * DMA_BK, wid, lane);
  } else {
    dma_stage<EXT, KMAJ, NW>(src, ld, k0, img, wid, lane);
  }
}
// 32x32x16 operand fragment (lane l: row/column base + (l & 31), k = kk + 8 (l >> 5) + 0..7)
// from the same two images.  k-row image: each 16-lane group g gathers columns
// base + 16 (g & 1) .. +15 of k-rows kk + 8 (g >> 1) + 0..3 and + 4..7 (two tr reads;
// tr_swz ignores k bit 2, so both share one swizzled column).
template <int EXT>
__device__ __forceinline__ bf16x8 dma_frag32(const bf16_t* img, bool kmajor_img, int base, int kk, int lane) {
  if (!kmajor_img) {
    const int r = base + (lane & 31);
    const int c = (kk >> 3) + (lane >> 5);
    return *reinterpret_cast<const bf16x8*>(img + r * DMA_BK + ((c ^ (r & 7)) << 3));
  }
  typedef __attribute__((ext_vector_type(4))) short s4;
  const int i16 = lane & 15, g4 = lane >> 4;
  const int k1 = kk + 8 * (g4 >> 1) + (i16 >> 2);
  const int col = base + 16 * (g4 & 1) + 4 * (i16 & 3);
  const int pcol = (((col >> 3) ^ tr_swz<EXT>(k1)) << 3) | (col & 7);
  const unsigned a0 = (unsigned)(uintptr_t)((__attribute__((address_space(3))) const bf16_t*)(img + k1 * EXT + pcol));
  s4 lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(a0));
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(a0), "n"(4 * EXT * 2));
  bf16x8 f;
  f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
  f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
  return f;
}
template <int EXT>
__device__ __forceinline__ bf16x8 frag_op32(const bf16_t* img, bool kmajor_img, int base, int kk, int lane) {
  if constexpr (EXT > 64) {
    if (kmajor_img) return dma_frag32<64>(img + (base >> 6) * 64 * DMA_BK, true, base & 63, kk, lane);
  }
  return dma_frag32<EXT>(img, kmajor_img, base, kk, lane);
}

template <int EXT>
__device__ __forceinline__ bf16x8 frag_op(const bf16_t* img, bool kmajor_img, int base, int kk, int lane) {
  if constexpr (EXT > 64) {
    if (kmajor_img) return dma_frag<64>(img + (base >> 6) * 64 * DMA_BK, true, base & 63, kk, lane);
  }
  return dma_frag<EXT>(img, kmajor_img, base, kk, lane);
}

template <int EXT>
__device__ __forceinline__ void dma_stage_rt(bool kmaj, const bf16_t* src, long ld, int k0, bf16_t* img, int wid,
                                             int lane) {
  if (kmaj) stage_op<EXT, true>(src, ld, k0, img, wid, lane);
  else stage_op<EXT, false>(src, ld, k0, img, wid, lane);
}

// The same for a K-tile that only has `kv` (= 32) valid k: lanes whose 16-byte
// piece lies past it issue nothing (EXEC-masked), so no load leaves the operand;
// the stale LDS they leave is never read (the MFMA loop stops at kv).
template <int EXT>
__device__ __forceinline__ void dma_stage_tail(bool kmaj, const bf16_t* src, long ld, int k0, int kv, bf16_t* img,
                                               int wid, int lane);
template <int EXT>
__device__ __forceinline__ void dma_stage_tail_rt(bool kmaj, const bf16_t* src, long ld, int k0, int kv, bf16_t* img,
                                                  int wid, int lane) {
  if constexpr (EXT > 64) {
    if (kmaj) {
#pragma unroll
      for (int h = 0; h < EXT / 64; ++h)
        dma_stage_tail<64>(true, src + h * 64, ld, k0, kv, img + h * 64 * DMA_BK, wid, lane);
      return;
    }
  }
  dma_stage_tail<EXT>(kmaj, src, ld, k0, kv, img, wid, lane);
}
template <int EXT>
__device__ __forceinline__ void dma_stage_tail(bool kmaj, const bf16_t* src, long ld, int k0, int kv, bf16_t* img,
                                               int wid, int lane) {
  constexpr int IPW = EXT / 32;
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int ins = wid * IPW + i;
    const int p = ins * 64 + lane;
    const bf16_t* gp;
    bool ok;
    if (!kmaj) {
      const int r = p >> 3, c = (p & 7) ^ (r & 7);
      gp = src + (long)r * ld + k0 + c * 8;
      ok = c * 8 < kv;
    } else {
      constexpr int CPR = EXT / 8;
      const int kr = p / CPR, cm = (p % CPR) ^ tr_swz<EXT>(kr);
      gp = src + (long)(k0 + kr) * ld + cm * 8;
      ok = kr < kv;
    }
    if (ok)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gp,
                                       (__attribute__((address_space(3))) void*)(img + ins * 512), 16, 0, 0);
  }
}

// Wait until at most `pend` K-tiles (LPW LDS-DMA instructions each, per wave)
// issued after the one about to be read are still in flight, then barrier.
// P is the ring's maximum (S - 2); the count must be an immediate, hence the
// unrolled chain.  Waiting for exactly what is needed keeps the ring's tail
// overlapped too (a plain vmcnt(0) there drains it S - 2 tiles early).
template <int LPW, int P>
__device__ __forceinline__ void dma_wait_barrier(int pend) {
  if constexpr (P > 0) {
    if (pend >= P) {
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(P * LPW) : "memory");
      return;
    }
    dma_wait_barrier<LPW, P - 1>(pend);
  } else {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
}

// R = 64-deep K sub-tiles per ring slot (one barrier per R sub-tiles): small
// tiles do too little MFMA work per barrier at R = 1 (a 32 x 32 tile: 2 MFMAs
// per wave between barriers; the wait / barrier / ds_read latency chain then
// sets the K loop's pace, ~300 cycles per 64-deep K-tile on one workgroup/CU).
// MF = 32: every wave's TM x TN sub-tiles are 32 x 32 (v_mfma_f32_32x32x16_bf16): half
// the LDS fragment traffic per FLOP, and the vectorised epilogue only.
template <int WM, int WN, int TM, int TN, bool AT, bool BT, int S, int R = 1, int MF = 16>
__global__ void __launch_bounds__(64 * WM * WN) gemm_dma_kernel(GemmArgs g, int tiles_n, int splits, int kchunk,
                                                                float* __restrict__ ws, unsigned* counters, int vec,
                                                                int group_m) {
  constexpr int NW = WM * WN;             // waves: 4, or 8 (two per SIMD) for the 128 x 128+ tiles
  constexpr int BM = WM * TM * MF, BN = WN * TN * MF, BK = DMA_BK;
  constexpr int SUB = (BM + BN) * BK;     // elements of one 64-deep sub-tile (A image then B image)
  constexpr int STAGE = SUB * R;          // elements of one ring slot
  constexpr int LPW = (BM + BN) / (8 * NW) * R;  // glds per wave per slot
  static_assert((S - 2) * LPW <= 63, "vmcnt range");
  __shared__ __attribute__((aligned(16))) bf16_t smem[S * STAGE];
  const int nwg = gridDim.x;
  int bid = blockIdx.x;
  {
    const int xcd = bid % 8, q = nwg / 8, rr = nwg % 8;
    bid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
  }
  int tmi = bid / tiles_n, tni = bid % tiles_n;
  if (group_m > 1) {
    // row-groups of group_m tiles, column-major inside a group: an XCD's contiguous
    // run of tiles is then a near-square block, so the operand panels it fetches
    // from beyond its L2 per K-tile shrink (2048 x 2048 / 128 x 128: 288 -> 192 KB)
    const int tiles_m = nwg / tiles_n, gsz = group_m * tiles_n, grp = bid / gsz, f = grp * group_m;
    const int gm = min(group_m, tiles_m - f), t = bid - grp * gsz;
    tmi = f + t % gm;
    tni = t / gm;
  }
  const int tm0 = tmi * BM, tn0 = tni * BN, z = blockIdx.z;
  const bf16_t* Ab = static_cast<const bf16_t*>(g.A) + zoff(g, z, g.sA, g.sA2) + (AT ? (long)tm0 : (long)tm0 * g.lda);
  const bf16_t* Bb = static_cast<const bf16_t*>(g.B) + zoff(g, z, g.sB, g.sB2) + (BT ? (long)tn0 : (long)tn0 * g.ldb);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int split = blockIdx.y;
  const int kbeg = split * kchunk;
  const int nkt = (min(g.K, kbeg + kchunk) - kbeg) / (BK * R);  // host: kchunk % (64 R) == 0

  using acc_t = typename std::conditional<MF == 32, f32x16, f32x4>::type;
  acc_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < (MF == 32 ? 16 : 4); ++e) acc[i][j][e] = 0.f;

  auto issue = [&](int kt) {
    bf16_t* st = smem + (kt % S) * STAGE;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int k0 = kbeg + (kt * R + r) * BK;
      stage_op<BM, AT, NW>(Ab, g.lda, k0, st + r * SUB, wid, lane);
      stage_op<BN, BT, NW>(Bb, g.ldb, k0, st + r * SUB + BM * BK, wid, lane);
    }
  };
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nkt) issue(s);
  for (int kt = 0; kt < nkt; ++kt) {
    // slot kt has landed once at most the slots issued after it are pending
    // (per wave), and every wave's share once all passed the barrier
    dma_wait_barrier<LPW, S - 2>(min(S - 2, nkt - 1 - kt));
    // refill the slot consumed in iteration kt-1 (all waves are past it)
    if (kt + S - 1 < nkt) issue(kt + S - 1);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const bf16_t* As = smem + (kt % S) * STAGE + r * SUB;
      const bf16_t* Bs = As + BM * BK;
      if constexpr (MF == 32) {
#pragma unroll
        for (int kk = 0; kk < BK; kk += 16) {
          bf16x8 af[TM], bfr[TN];
#pragma unroll
          for (int i = 0; i < TM; ++i) af[i] = frag_op32<BM>(As, AT, (wm * TM + i) * 32, kk, lane);
#pragma unroll
          for (int j = 0; j < TN; ++j) bfr[j] = frag_op32<BN>(Bs, BT, (wn * TN + j) * 32, kk, lane);
          if constexpr (AT || BT) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(af[i]));
#pragma unroll
            for (int j = 0; j < TN; ++j) asm volatile("" : "+v"(bfr[j]));
          }
#pragma unroll
          for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j) acc[i][j] = mfma32x32x16(af[i], bfr[j], acc[i][j]);
        }
      } else {
#pragma unroll
      for (int kk = 0; kk < BK; kk += 32) {
        bf16x8 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = frag_op<BM>(As, AT, (wm * TM + i) * 16, kk, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[j] = frag_op<BN>(Bs, BT, (wn * TN + j) * 16, kk, lane);
        if constexpr (AT || BT) {
          // asm tr reads retired; the empty asm ties every fragment to the wait so
          // no MFMA can be scheduled ahead of it
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
          for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(af[i]));
#pragma unroll
          for (int j = 0; j < TN; ++j) asm volatile("" : "+v"(bfr[j]));
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(af[i], bfr[j], acc[i][j]);
      }
      }
    }
  }
  __syncthreads();
  static_assert((BM * (BN + 4) + 4) * 4 <= S * STAGE * 2, "output image fits the staging ring");
  if constexpr (MF == 32) {
    // launched only where the vectorised epilogue applies (host)
    gemm_finish_vec32<BM, BN, TM, TN, 64 * NW>(g, acc, tm0, tn0, z, wm, wn, lane, tid, splits, split,
                                               (long)z * gridDim.x + bid, ws, counters, reinterpret_cast<float*>(smem));
  } else if constexpr (NW != 4) {
    // 8-wave tiles are launched only where the vectorised epilogue applies (host)
    gemm_finish_vec<BM, BN, TM, TN, 64 * NW>(g, acc, tm0, tn0, z, wm, wn, lane, tid, splits, split,
                                             (long)z * gridDim.x + bid, ws, counters, reinterpret_cast<float*>(smem));
  } else if (vec) {
    gemm_finish_vec<BM, BN, TM, TN>(g, acc, tm0, tn0, z, wm, wn, lane, tid, splits, split,
                                    (long)z * gridDim.x + bid, ws, counters, reinterpret_cast<float*>(smem));
  } else if constexpr (TM * TN >= 16) {
    gemm_finish_lds<BM, BN, TM, TN>(g, acc, tm0, tn0, z, wm, wn, lane, tid, splits, split,
                                    (long)z * gridDim.x + bid, ws, counters, reinterpret_cast<float*>(smem));
  } else {
    gemm_finish<BM, BN, TM, TN>(g, acc, tm0, tn0, z, wid, wm, wn, lane, tid, splits, split, (long)z * gridDim.x + bid,
                                ws, counters, reinterpret_cast<int*>(smem));
  }
}


// ---------------------------------------------------------------------------
// Grouped LDS-DMA GEMM: up to GROUP_MAX independent problems (e.g. a layer's
// weight gradient h^T dz and its input gradient dz W^T, which both only need
// dz) in ONE launch -- one grid whose workgroups pick their problem from a
// prefix table, so the two GEMMs' tiles run side by side on the CUs instead of
// the second queueing behind the first's tail, and one launch gap is saved.
// 32x32 tiles, no K split, K % 32 == 0 (a 32-deep tail tile is loaded with
// EXEC-masked DMA); operand layouts are per-problem runtime flags.
constexpr int GROUP_MAX = 4;
struct GemmGroup {
  GemmArgs g[GROUP_MAX];
  int tiles_n[GROUP_MAX];
  int start[GROUP_MAX + 1];
  int n;
  // per-problem split-K (1 = none): a long-K problem (e.g. an input gradient
  // with K = d_ff next to its K = tokens weight gradient) would otherwise be the
  // group's long pole; its slices combine through gemm_finish's slabs/tickets
  int splits[GROUP_MAX];
  long wsoff[GROUP_MAX];
  int cntoff[GROUP_MAX];
  int vec[GROUP_MAX];   // epi_vec_ok per problem
  float* ws;
  unsigned* counters;
};

template <int S, bool TAIL, int TM = 1, int TN = 1>
__global__ void __launch_bounds__(256) gemm_dma_group_kernel(GemmGroup G) {
  constexpr int WM = 2, WN = 2;
  constexpr int BM = WM * TM * 16, BN = WN * TN * 16, BK = DMA_BK;
  constexpr int STAGE = (BM + BN) * BK;
  constexpr int LPW = BM / 32 + BN / 32;
  __shared__ __attribute__((aligned(16))) bf16_t smem[S * STAGE];
  const int nwg = gridDim.x;
  int bid = blockIdx.x;
  {
    const int xcd = bid % 8, q = nwg / 8, rr = nwg % 8;
    bid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
  }
  int p = 0;
#pragma unroll
  for (int t = 1; t < GROUP_MAX; ++t)
    if (t < G.n && bid >= G.start[t]) p = t;
  const GemmArgs& g = G.g[p];
  const int tn = G.tiles_n[p], sp = G.splits[p];
  const int tiles_p = (g.M / BM) * tn;
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int local = bid - G.start[p];
  const int tile = local % tiles_p, split = local / tiles_p;
  const int tm0 = (tile / tn) * BM, tn0 = (tile % tn) * BN;
  const int kchunk = g.K / sp, k0 = split * kchunk;   // sp > 1: kchunk % BK == 0 (host)
  const bool at = g.a_trans, bt = g.b_trans;
  const bf16_t* Ab = static_cast<const bf16_t*>(g.A) + (at ? (long)tm0 : (long)tm0 * g.lda);
  const bf16_t* Bb = static_cast<const bf16_t*>(g.B) + (bt ? (long)tn0 : (long)tn0 * g.ldb);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int nkt = (kchunk + BK - 1) / BK;  // K % 32 == 0: the last tile may hold 32 valid k
  auto issue = [&](int kt) {
    bf16_t* st = smem + (kt % S) * STAGE;
    const int kv = kchunk - kt * BK;
    if (!TAIL || kv >= BK) {
      dma_stage_rt<BM>(at, Ab, g.lda, k0 + kt * BK, st, wid, lane);
      dma_stage_rt<BN>(bt, Bb, g.ldb, k0 + kt * BK, st + BM * BK, wid, lane);
    } else {
      dma_stage_tail_rt<BM>(at, Ab, g.lda, k0 + kt * BK, kv, st, wid, lane);
      dma_stage_tail_rt<BN>(bt, Bb, g.ldb, k0 + kt * BK, kv, st + BM * BK, wid, lane);
    }
  };
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nkt) issue(s);
  for (int kt = 0; kt < nkt; ++kt) {
    if (kt + S - 2 < nkt) {
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"((S - 2) * LPW) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    if (kt + S - 1 < nkt) issue(kt + S - 1);
    const bf16_t* As = smem + (kt % S) * STAGE;
    const bf16_t* Bs = As + BM * BK;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      if (TAIL && kt * BK + kk >= kchunk) break;  // half tile (uniform)
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[i] = at ? frag_op<BM>(As, true, (wm * TM + i) * 16, kk, lane)
                   : frag_op<BM>(As, false, (wm * TM + i) * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[j] = bt ? frag_op<BN>(Bs, true, (wn * TN + j) * 16, kk, lane)
                    : frag_op<BN>(Bs, false, (wn * TN + j) * 16, kk, lane);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // asm tr reads retired (see gemm_dma_kernel)
#pragma unroll
      for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(af[i]));
#pragma unroll
      for (int j = 0; j < TN; ++j) asm volatile("" : "+v"(bfr[j]));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(af[i], bfr[j], acc[i][j]);
    }
  }
  __syncthreads();
  if (G.vec[p]) {
    gemm_finish_vec<BM, BN, TM, TN>(g, acc, tm0, tn0, 0, wm, wn, lane, tid, sp, split, tile,
                                    sp > 1 ? G.ws + G.wsoff[p] : nullptr, sp > 1 ? G.counters + G.cntoff[p] : nullptr,
                                    reinterpret_cast<float*>(smem));
  } else if constexpr (TM * TN >= 16) {
    gemm_finish_lds<BM, BN, TM, TN>(g, acc, tm0, tn0, 0, wm, wn, lane, tid, sp, split, tile,
                                    sp > 1 ? G.ws + G.wsoff[p] : nullptr, sp > 1 ? G.counters + G.cntoff[p] : nullptr,
                                    reinterpret_cast<float*>(smem));
  } else {
    gemm_finish<BM, BN, TM, TN>(g, acc, tm0, tn0, 0, wid, wm, wn, lane, tid, sp, split, tile,
                                sp > 1 ? G.ws + G.wsoff[p] : nullptr, sp > 1 ? G.counters + G.cntoff[p] : nullptr,
                                reinterpret_cast<int*>(smem));
  }
}

// ---------------------------------------------------------------------------
// The W pass in ONE launch (transformer stages, models/transformer.py weight_grads):
// every deferred weight-gradient GEMM of a step, dW_p = A_p^T B_p with both operands
// token-major (A_p = a layer's input [T][M_p], B_p = its output gradient [T][N_p],
// K = T tokens), AdamW in the vectorised epilogue.  Workgroups pick their problem from a
// prefix table in DEVICE memory (17 GemmArgs do not fit a kernel-argument block); the
// main loop is gemm_dma_kernel's for two transposed operands (LDS-DMA ring, counted
// vmcnt, ds_read_b64_tr_b16 fragments).  Replaces 17 launches round-robin over the
// microbatch streams: the GEMMs' tiles fill the chip side by side instead of each
// stream's small GEMMs queueing behind its large ones, and the AdamW epilogues of one
// problem overlap the main loops of the others.
constexpr int WP_MAX = 40;
struct GemmWTable {
  int n, total;
  int start[WP_MAX + 1];
  int tiles_n[WP_MAX];
  int splits[WP_MAX];
  long wsoff[WP_MAX];
  int cntoff[WP_MAX];
  float* ws;
  unsigned* counters;
  GemmArgs g[WP_MAX];
};

template <int TM, int TN, int MF, int S>
__global__ void __launch_bounds__(256) gemm_wpass_kernel(const GemmWTable* __restrict__ T) {
  constexpr int WM = 2, WN = 2, NW = 4;
  constexpr int BM = WM * TM * MF, BN = WN * TN * MF, BK = DMA_BK;
  constexpr int STAGE = (BM + BN) * BK;
  constexpr int LPW = (BM + BN) / (8 * NW);   // glds per wave per K-tile
  static_assert((S - 2) * LPW <= 63, "vmcnt range");
  __shared__ __attribute__((aligned(16))) bf16_t smem[S * STAGE];
  const int nwg = gridDim.x;
  int bid = blockIdx.x;
  {
    const int xcd = bid % 8, q = nwg / 8, rr = nwg % 8;
    bid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
  }
  // the problem: scalar loads of the prefix table (wave-uniform address)
  const int n = T->n;
  int p = 0;
  for (int t = 1; t < n; ++t)
    if (bid >= T->start[t]) p = t;
  p = __builtin_amdgcn_readfirstlane(p);
  const GemmArgs& g = T->g[p];
  const int tn = T->tiles_n[p], sp = T->splits[p];
  const int tiles_p = (g.M / BM) * tn;
  const int local = bid - T->start[p];
  const int tile = local % tiles_p, split = local / tiles_p;
  const int tm0 = (tile / tn) * BM, tn0 = (tile % tn) * BN;
  const int kchunk = g.K / sp, kbeg = split * kchunk;   // host: kchunk % 64 == 0
  const bf16_t* Ab = static_cast<const bf16_t*>(g.A) + tm0;   // "km": A[k][m] at k * lda + m
  const bf16_t* Bb = static_cast<const bf16_t*>(g.B) + tn0;   // "kn": B[k][n] at k * ldb + n
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int nkt = kchunk / BK;
  using acc_t = typename std::conditional<MF == 32, f32x16, f32x4>::type;
  acc_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < (MF == 32 ? 16 : 4); ++e) acc[i][j][e] = 0.f;
  auto issue = [&](int kt) {
    bf16_t* st = smem + (kt % S) * STAGE;
    const int k0 = kbeg + kt * BK;
    stage_op<BM, true, NW>(Ab, g.lda, k0, st, wid, lane);
    stage_op<BN, true, NW>(Bb, g.ldb, k0, st + BM * BK, wid, lane);
  };
#pragma unroll
  for (int s2 = 0; s2 < S - 1; ++s2)
    if (s2 < nkt) issue(s2);
  for (int kt = 0; kt < nkt; ++kt) {
    dma_wait_barrier<LPW, S - 2>(min(S - 2, nkt - 1 - kt));
    if (kt + S - 1 < nkt) issue(kt + S - 1);
    const bf16_t* As = smem + (kt % S) * STAGE;
    const bf16_t* Bs = As + BM * BK;
    if constexpr (MF == 32) {
#pragma unroll
      for (int kk = 0; kk < BK; kk += 16) {
        bf16x8 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = frag_op32<BM>(As, true, (wm * TM + i) * 32, kk, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[j] = frag_op32<BN>(Bs, true, (wn * TN + j) * 32, kk, lane);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // asm tr reads retired (gemm_dma_kernel)
#pragma unroll
        for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(af[i]));
#pragma unroll
        for (int j = 0; j < TN; ++j) asm volatile("" : "+v"(bfr[j]));
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma32x32x16(af[i], bfr[j], acc[i][j]);
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < BK; kk += 32) {
        bf16x8 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = frag_op<BM>(As, true, (wm * TM + i) * 16, kk, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[j] = frag_op<BN>(Bs, true, (wn * TN + j) * 16, kk, lane);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(af[i]));
#pragma unroll
        for (int j = 0; j < TN; ++j) asm volatile("" : "+v"(bfr[j]));
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(af[i], bfr[j], acc[i][j]);
      }
    }
  }
  __syncthreads();
  static_assert((BM * (BN + 4) + 4) * 4 <= S * STAGE * 2, "output image fits the staging ring");
  float* const wsp = sp > 1 ? T->ws + T->wsoff[p] : nullptr;
  unsigned* const cnt = sp > 1 ? T->counters + T->cntoff[p] : nullptr;
  if constexpr (MF == 32)
    gemm_finish_vec32<BM, BN, TM, TN>(g, acc, tm0, tn0, 0, wm, wn, lane, tid, sp, split, tile, wsp, cnt,
                                      reinterpret_cast<float*>(smem));
  else
    gemm_finish_vec<BM, BN, TM, TN>(g, acc, tm0, tn0, 0, wm, wn, lane, tid, sp, split, tile, wsp, cnt,
                                    reinterpret_cast<float*>(smem));
}

// Exact-slice depth: K-tiles a slice may hold in registers (~128 VGPRs of
// staged bf16 operands) and in one LDS image (<= 160 KB).
template <int WM, int WN, int TM, int TN, int BK>
constexpr int exact_depth() {
  using T = Tile<WM, WN, TM, TN, BK>;
  constexpr int dr = 128 / (4 * (T::A_PER_T + T::B_PER_T));
  constexpr int dl = (81920 / (T::BM + T::BN) - 8) / BK;
  constexpr int d = dr < dl ? dr : dl;
  return d >= 16 ? 16 : (d >= 8 ? 8 : (d >= 4 ? 4 : 2));
}
static int g_exact_pre = 0;  // jdt_gemm_set_exact(pre): force the exact slice depth (tuning sweeps); 0 = auto

constexpr int kPreMax = 4;      // K-tiles a preloading slice holds in registers
static bool g_gemm_no_preload = false;  // jdt_gemm_set_preload(0): pipelined path only (A/B tests)

static bool g_epi_vec = true;  // jdt_gemm_set_epi_vec(0): per-element epilogue (A/B tests)
static long g_epi_vec_min = 0;  // jdt_gemm_set_epi_vec_min(n): vectorised epilogue only from n outputs

template <int WM, int WN, int TM, int TN, int BK>
static int launch_cfg(const GemmArgs& g, int batch, int splits, float* ws, long ws_floats, unsigned* counters,
                      long n_counters, hipStream_t st) {
  using T = Tile<WM, WN, TM, TN, BK>;
  const int tiles_m = (g.M + T::BM - 1) / T::BM, tiles_n = (g.N + T::BN - 1) / T::BN;
  const long tiles = (long)tiles_m * tiles_n * batch;
  const int ktiles = (g.K + BK - 1) / BK;
  // vector loads need 16-byte aligned rows: bf16 ld % 8, f32 ld % 4, aligned base
  auto vec_ok = [](const void* p, long ld, int f32) {
    return ((reinterpret_cast<uintptr_t>(p) & 15) == 0) && (f32 ? (ld % 4 == 0) : (ld % 8 == 0));
  };
  const int va = vec_ok(g.A, g.lda, g.a_f32), vb = vec_ok(g.B, g.ldb, g.b_f32);
  const int vec = g_epi_vec && (long)g.M * g.N * batch >= g_epi_vec_min && epi_vec_ok(g, batch);
  // Exact path: bf16 operands, every tile interior, K a whole number of
  // K-tiles split into slices of exactly `pre` (power of two <= register
  // depth) -- straight-line kernels with one global round trip per slice.
  if (splits < 0 && !g_gemm_no_preload && !g.a_f32 && !g.b_f32 && va && vb && g.M % T::BM == 0 &&
      g.N % T::BN == 0 && g.K % BK == 0) {
    constexpr int depth = exact_depth<WM, WN, TM, TN, BK>();
    int pre = depth;
    while (pre > 1 && ktiles % pre) pre >>= 1;
    if (g_exact_pre > 0 && g_exact_pre <= depth && ktiles % g_exact_pre == 0) pre = g_exact_pre;
    const int sp = ktiles / pre;
    const bool ws_ok = sp == 1 || (ws && counters && tiles * sp * T::BM * T::BN <= ws_floats && tiles <= n_counters);
    // a K split pays a slab round trip + combine: only while the grid is not already full
    const bool split_ok = sp == 1 || g_exact_pre > 0 || tiles * sp <= 256;
    if (pre >= 2 && sp <= 16 && ws_ok && split_ok) {
      dim3 egrid(tiles_m * tiles_n, sp, batch);
      const int ekchunk = pre * BK;
#define JDT_GEMM_EXACT(P)                                                                                         \
  case P:                                                                                                        \
    hipLaunchKernelGGL((gemm_kernel<WM, WN, TM, TN, BK, false, false, (P <= depth ? P : depth), true>), egrid,   \
                       dim3(256), 0, st, g,                                                                      \
                       tiles_n, va, vb, sp, ekchunk, ws, counters, vec);                                         \
    return HIP_LAUNCH_CHECK();
      switch (pre) {
        JDT_GEMM_EXACT(2)
        JDT_GEMM_EXACT(4)
        JDT_GEMM_EXACT(8)
        JDT_GEMM_EXACT(16)
        default: break;
      }
#undef JDT_GEMM_EXACT
    }
  }
  if (splits < 0) {
    // Small GEMMs here are latency-bound on the K loop (one global round trip
    // per K-tile): split K until the grid covers ~all CUs, <= 16 slices,
    // each slice at least one K-tile.
    // With the preload path a slice costs one round trip whatever its length,
    // so split only to fill the CUs (<= ~256 workgroups).
    splits = 1;
    while (splits < 16 && tiles * splits * 2 <= 256 && ktiles >= splits * 2) splits *= 2;
    while (splits < 16 && (ktiles + splits - 1) / splits > kPreMax && tiles * splits * 2 <= 512) splits *= 2;
  }
  if (splits > ktiles) splits = ktiles;
  if (splits < 1) splits = 1;
  if (splits > 1 && (!ws || !counters || tiles * splits * T::BM * T::BN > ws_floats || tiles > n_counters))
    splits = 1;
  const int kchunk = ((ktiles + splits - 1) / splits) * BK;
  splits = (g.K + kchunk - 1) / kchunk;
  dim3 grid(tiles_m * tiles_n, splits, batch);
  const bool pre = kchunk / BK <= kPreMax && !g_gemm_no_preload;
#define JDT_GEMM_LAUNCH(AF, BF)                                                                                  \
  do {                                                                                                           \
    if (pre)                                                                                                     \
      hipLaunchKernelGGL((gemm_kernel<WM, WN, TM, TN, BK, AF, BF, kPreMax>), grid, dim3(256), 0, st, g, tiles_n, \
                         va, vb, splits, kchunk, ws, counters, vec);                                             \
    else                                                                                                         \
      hipLaunchKernelGGL((gemm_kernel<WM, WN, TM, TN, BK, AF, BF, 0>), grid, dim3(256), 0, st, g, tiles_n, va,   \
                         vb, splits, kchunk, ws, counters, vec);                                                 \
  } while (0)
  if (g.a_f32 && g.b_f32) JDT_GEMM_LAUNCH(true, true);
  else if (g.a_f32)       JDT_GEMM_LAUNCH(true, false);
  else if (g.b_f32)       JDT_GEMM_LAUNCH(false, true);
  else                    JDT_GEMM_LAUNCH(false, false);
#undef JDT_GEMM_LAUNCH
  return HIP_LAUNCH_CHECK();
}


static bool g_gemm_no_dma = false;  // jdt_gemm_set_dma(0): register-staged kernels only (A/B tests)
static int g_group_split = 1;  // jdt_gemm_set_group_split(0): no split-K inside grouped launches (A/B tests)

// LDS ring depth 3 (one K-tile in flight across each barrier).  Deeper rings
// cost resident workgroups per CU (qkv 512x1536x512: 9.8 us with 8 stages vs
// 6.8 with 3); a plain double buffer (2) is as fast for an isolated GEMM but
// 4-8 % slower inside the transformer / GPipe steps, where the operands are
// colder (tools/bench_gemm.py, bench.py --strategy pp).
template <int BM, int BN>
constexpr int dma_stages() { return 3; }

// (Measured and dropped, BENCH_NOTES.md: an 8-stage "deep" ring for grids of <= 1
// workgroup per CU -- no faster in isolation, slower in-model; and software-
// pipelined fragment reads (both 32-deep halves of a slot issued up front, counted
// lgkmcnt) -- within noise: the K loop waits on the global->LDS ring, not on LDS.)
static int g_group_m = -1;  // jdt_gemm_set_group_m(G): force tile row-groups of G (0 = row-major), -1 = table
static int g_dma_r = -1;  // jdt_gemm_set_r(r): force r 64-deep sub-tiles per ring slot (sweeps); -1 auto
// R > 1 slots: 3 of them within 96 KB (and the vmcnt immediate range)
template <int BM, int BN>
constexpr bool r_ok(int r) { return r == 1 || ((BM + BN) * DMA_BK * 2 * 3 * r <= 96 * 1024 && (BM / 32 + BN / 32) * r <= 63); }

// MF: MFMA sub-tile (16: 16x16x32, 32: 32x32x16); SD: ring depth (0 = dma_stages)
template <int WM, int WN, int TM, int TN, int MF = 16, int SD = 0>
static int launch_dma(const GemmArgs& g, int batch, int splits, float* ws, long ws_floats, unsigned* counters,
                      long n_counters, hipStream_t st, int r_pref = 1, int gm_pref = 0) {
  constexpr int BM = WM * TM * MF, BN = WN * TN * MF;
  constexpr int SR = SD > 0 ? SD : dma_stages<BM, BN>();
  if (g.M % BM || g.N % BN) return 1;
  const int tiles_n = g.N / BN;
  const long tiles = (long)(g.M / BM) * tiles_n * batch;
  int sp = splits;
  if (sp < 0) {
    // Measured (tools/bench_gemm.py sweeps): many small workgroups per CU hide
    // the load latency better than a split-K combine (whose last-arriving slice
    // reads every slab serially); split only while the grid has < 2 workgroups
    // per CU, keeping slices >= 8 K-tiles.
    sp = 1;
    while (sp < 16 && tiles * sp < 512 && (g.K / (2 * sp)) % DMA_BK == 0 && g.K / (2 * sp) >= 8 * DMA_BK) sp *= 2;
  }
  if (sp < 1 || g.K % sp || (g.K / sp) % DMA_BK) return 1;
  if (sp > 1 && (!ws || !counters || tiles * sp * BM * BN > ws_floats || tiles > n_counters)) sp = 1;
  const int kchunk = g.K / sp;
  dim3 grid((g.M / BM) * tiles_n, sp, batch);
  const bool at = g.a_trans, bt = g.b_trans;
  // 32 x 32 tiles keep the per-element epilogue: the LDS round trip and barrier
  // cost more than the narrow stores on those small outputs (in-model A/B,
  // tools/gpu_r2_ab_epi.sh: microbatch-loop transformer 3.07 ms vec vs 2.98)
  const int vec = g_epi_vec && BM * BN >= 2048 && (long)g.M * g.N * batch >= g_epi_vec_min && epi_vec_ok(g, batch);
  if ((WM * WN != 4 || MF == 32) && !epi_vec_ok(g, batch)) return 1;  // 8-wave / 32x32 tiles: vectorised epilogue only
  // sub-tiles per ring slot: g_dma_r forces (sweeps), else 1
  int R = g_dma_r > 0 ? g_dma_r : r_pref;
  const int gm = g_group_m >= 0 ? g_group_m : gm_pref;
  while (R > 1 && (kchunk / DMA_BK) % R) R >>= 1;
  if (R > 1 && !r_ok<BM, BN>(R)) R = 1;
#define JDT_DMA_S(A_, B_, S_, R_)                                                                                 \
  hipLaunchKernelGGL((gemm_dma_kernel<WM, WN, TM, TN, A_, B_, S_, R_, MF>), grid, dim3(64 * WM * WN), 0, st, g,    \
                     tiles_n, sp, kchunk, ws, counters, vec, gm)
#define JDT_DMA(A_, B_)                                                   \
  do {                                                                    \
    if constexpr (r_ok<BM, BN>(4)) {                                      \
      if (R == 4) { JDT_DMA_S(A_, B_, 3, 4); break; }                     \
    }                                                                     \
    if constexpr (r_ok<BM, BN>(2)) {                                      \
      if (R == 2) { JDT_DMA_S(A_, B_, 3, 2); break; }                     \
    }                                                                     \
    JDT_DMA_S(A_, B_, SR, 1);                                             \
  } while (0)
  if (!at && !bt) JDT_DMA(false, false);
  else if (!at && bt) JDT_DMA(false, true);
  else if (at && !bt) JDT_DMA(true, false);
  else JDT_DMA(true, true);
#undef JDT_DMA
#undef JDT_DMA_S
  return HIP_LAUNCH_CHECK();
}

// LDS-DMA path for bf16 operands: returns 1 if the shape / layout is outside
// its envelope (caller falls back to the register-staged kernels).
// Measured tile choices (tools/bench_gemm.py --cfg C --r R sweeps on MI355X,
// profiles/r2_gemm_tile_sweep.txt): the 2048-token transformer shapes.  The
// 512-row entries the isolated sweep also favoured were dropped: inside the
// microbatch-loop transformer step (colder operands, neighbouring kernels) they
// measured 2 % slower than the heuristic (tools/gpu_r2_ab_tune.sh).
// Tile ORDER (gm): long-K problems with small tiles fetch the operand panels of
// their whole tile row from beyond the XCD's L2 every K-tile; ordering the tiles
// in row-groups of gm (column-major inside a group) makes each XCD's contiguous
// run of tiles a near-square block (qkv dW 19.9 -> 16.3 us at gm = 8; no effect
// on the 2048 x 2048 short-K shapes).  cfg 15 / 16: 8-wave 128 x 128 tiles.
// {M, N, K, a_trans, b_trans, cfg, R, gm}.
struct GemmTune { int M, N, K, at, bt, cfg, r, gm; };
static const GemmTune kGemmTune[] = {
    {2048, 512, 2048, 0, 1, 10, 2, 0},   // fc2 fwd                   14.41 (13.78)
    {512, 2048, 2048, 1, 1, 10, 1, 8},   // fc1 / head dW             17.46 (16.26)
    {2048, 2048, 512, 0, 1, 15, 1, 0},   // fc1 / head fwd            10.37 (11.02)
    {2048, 2048, 512, 0, 0, 16, 1, 0},   // fc2 dX                    10.16 (9.91)
    {2048, 512, 2048, 0, 0, 10, 2, 0},   // fc1 / head dX             12.00 (10.98)
    {2048, 512, 2048, 1, 1, 10, 2, 0},   // fc2 dW                    15.48 (16.53)
    {512, 1536, 2048, 1, 1, 10, 1, 8},   // qkv dW                    16.28 (16.09)
    {512, 512, 2048, 1, 1, 13, 2, 0},    // out dW                    10.41 (15.46)
    {256, 1536, 512, 0, 1, 10, 2, 0},    // qkv fwd (hybrid, 256 rows) 5.55 (5.60)
    {256, 512, 2048, 0, 1, 13, 2, 0},    // fc2 fwd (hybrid)          8.38 (9.84)
    // round 3: 512-row (one microbatch of 4 sequences) and qkv shapes, from the cfg x split-K
    // sweeps (profiles/r3_gemm_mfma32_sweep.txt, r3_gemm_cfg_split_sweep.txt; previous
    // table / heuristic time in parentheses)
    {512, 2048, 512, 0, 1, 10, 1, 0},    // fc1 / head fwd, 512 rows   6.60 (10.76; cfg 20 7.52)
    {512, 2048, 512, 0, 0, 10, 1, 0},    // fc2 dX, 512 rows           5.95 (9.67; cfg 20 7.26)
    {512, 512, 2048, 0, 1, 10, 1, 0},    // fc2 fwd, 512 rows (split 4) 10.00 (11.41)
    {512, 512, 2048, 0, 0, 10, 1, 0},    // fc1 / head dX, 512 rows     9.42 (10.16)
    {512, 512, 1536, 0, 0, 10, 1, 0},    // qkv dX, 512 rows (as fc1 dX)
    {512, 2048, 512, 1, 1, 20, 1, 0},    // fc1 dW, 512 tokens         8.11 (9.80)
    {2048, 512, 512, 1, 1, 20, 1, 0},    // fc2 dW, 512 tokens         8.15 (9.92)
    {2048, 1536, 512, 0, 1, 26, 1, 0},   // qkv fwd (2048 rows)       11.87 (14.92)
    // round 6: the layer-major LM pass's 2048-row N = 512 GEMMs (the heuristic's 32 x 32
    // tiles; profiles/r6_s4_gemm_sweep.txt)
    {2048, 512, 512, 0, 1, 10, 1, 0},    // out fwd 2k                 6.55 (10.32)
    {2048, 512, 512, 0, 0, 10, 1, 0},    // out dX 2k                  5.92 (9.45)
    {2048, 512, 1536, 0, 0, 10, 1, 0},   // qkv dX 2k                 11.04 (16.78)
};
static bool g_gemm_tune = true;  // jdt_gemm_set_tune(0): heuristic only (A/B)

static int gemm_dma(const GemmArgs& g, int batch, int cfg, int splits, float* ws, long ws_floats, unsigned* counters,
                    long n_counters, hipStream_t st) {
  if (g_gemm_no_dma || g.a_f32 || g.b_f32 || g.K % DMA_BK) return 1;
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (!al(g.A) || !al(g.B) || g.lda % 8 || g.ldb % 8) return 1;
  if (batch > 1 && (g.sA % 8 || g.sB % 8 || g.sA2 % 8 || g.sB2 % 8)) return 1;
  int r_pref = 1, gm_pref = 0;
  if (cfg < 0 && g_gemm_tune && batch == 1 && splits < 0) {
    for (const GemmTune& t : kGemmTune)
      if (t.M == g.M && t.N == g.N && t.K == g.K && t.at == (g.a_trans != 0) && t.bt == (g.b_trans != 0)) {
        cfg = t.cfg;
        r_pref = t.r;
        gm_pref = t.gm;
        break;
      }
  }
  if (cfg < 0) {
    // 32x32 tiles up to ~4 workgroups per CU (up to 6 fit by LDS), then 64x64,
    // then 64x128 (tools/bench_gemm.py sweep on the transformer/MLP shapes)
    const long t32 = (long)(g.M / 32) * (g.N / 32) * batch;
    const long t64 = (long)(g.M / 64) * (g.N / 64) * batch;
    if (g.M % 32 || g.N % 32) return 1;
    if (g.M < 64 && g.N < 256) return 1;  // tiny: the register kernels' split-K preload is as good
    if (t32 > 512 && g.K >= 2048 && g.N % 64 == 0) cfg = 10;  // long K: 32x64 reuses more per load
    else if (t32 <= 1024 || g.M % 64 || g.N % 64) cfg = 13;
    else if (t64 <= 768 || g.N % 128) cfg = 11;
    else cfg = 12;
  }
  int rc = 1;
  switch (cfg) {
    case 10: return launch_dma<2, 2, 1, 2>(g, batch, splits, ws, ws_floats, counters, n_counters, st, r_pref, gm_pref);  // 32 x 64
    case 11: return launch_dma<2, 2, 2, 2>(g, batch, splits, ws, ws_floats, counters, n_counters, st, r_pref, gm_pref);  // 64 x 64
    case 12: return launch_dma<2, 2, 2, 4>(g, batch, splits, ws, ws_floats, counters, n_counters, st, r_pref, gm_pref);  // 64 x 128
    case 13: return launch_dma<2, 2, 1, 1>(g, batch, splits, ws, ws_floats, counters, n_counters, st, r_pref, gm_pref);  // 32 x 32
    case 14: return launch_dma<2, 2, 4, 4>(g, batch, splits, ws, ws_floats, counters, n_counters, st, r_pref, gm_pref);  // 128 x 128
    // 8 waves (two per SIMD: one wave's LDS reads / DMA issue under the other's MFMAs)
    case 15: rc = launch_dma<2, 4, 4, 2>(g, batch, splits, ws, ws_floats, counters, n_counters, st, 1, gm_pref); break;  // 128 x 128
    case 16: rc = launch_dma<4, 2, 2, 4>(g, batch, splits, ws, ws_floats, counters, n_counters, st, 1, gm_pref); break;  // 128 x 128
    case 17: rc = launch_dma<4, 2, 4, 4>(g, batch, splits, ws, ws_floats, counters, n_counters, st, 1, gm_pref); break;  // 256 x 128
    case 18: rc = launch_dma<2, 4, 4, 4>(g, batch, splits, ws, ws_floats, counters, n_counters, st, 1, gm_pref); break;  // 128 x 256
    // 32 x 32 x 16 MFMA sub-tiles (4 waves unless noted)
    case 20: rc = launch_dma<2, 2, 1, 1, 32>(g, batch, splits, ws, ws_floats, counters, n_counters, st, r_pref, gm_pref); break;  // 64 x 64
    case 21: rc = launch_dma<2, 2, 1, 1, 32, 4>(g, batch, splits, ws, ws_floats, counters, n_counters, st, 1, gm_pref); break;   // 64 x 64, 4-slot ring
    case 22: rc = launch_dma<2, 2, 2, 1, 32>(g, batch, splits, ws, ws_floats, counters, n_counters, st, r_pref, gm_pref); break;  // 128 x 64
    case 23: rc = launch_dma<2, 2, 1, 2, 32>(g, batch, splits, ws, ws_floats, counters, n_counters, st, r_pref, gm_pref); break;  // 64 x 128
    case 24: rc = launch_dma<2, 2, 2, 2, 32>(g, batch, splits, ws, ws_floats, counters, n_counters, st, 1, gm_pref); break;   // 128 x 128
    case 25: rc = launch_dma<2, 2, 2, 2, 32, 4>(g, batch, splits, ws, ws_floats, counters, n_counters, st, 1, gm_pref); break;  // 128 x 128, 4-slot
    case 26: rc = launch_dma<4, 2, 1, 2, 32>(g, batch, splits, ws, ws_floats, counters, n_counters, st, 1, gm_pref); break;   // 128 x 128, 8 waves
    case 27: rc = launch_dma<2, 2, 2, 1, 32, 4>(g, batch, splits, ws, ws_floats, counters, n_counters, st, 1, gm_pref); break;  // 128 x 64, 4-slot
    default: return 1;
  }
  // 8-wave tiles outside their envelope (shape, or rows not 16-byte aligned for the
  // vectorised epilogue): the 4-wave 64 x 128 tile
  if (rc == 1) rc = launch_dma<2, 2, 2, 4>(g, batch, splits, ws, ws_floats, counters, n_counters, st, 1, gm_pref);
  return rc;
}


// Grouped launch (see gemm_dma_group_kernel).  Returns 1 if any problem is
// outside the envelope (bf16, 16-byte aligned rows, M, N, K % 32 == 0, no
// batch) -- the caller then launches the problems one by one.
static int g_group_tile = 0;  // jdt_gemm_set_group_tile(t): force 32 / 64 / 128 tiles (sweeps); 0 = heuristic

template <int T>
static int group_plan(const GemmArgs* gs, int n, GemmGroup& G, float* ws, long ws_floats, unsigned* counters,
                      long n_counters) {
  G.n = n;
  G.ws = ws;
  G.counters = counters;
  int total = 0;
  long wsused = 0, cntused = 0;
  for (int p = 0; p < n; ++p) {
    const GemmArgs& g = gs[p];
    if (g.M % T || g.N % T) return -1;
    G.g[p] = g;
    G.tiles_n[p] = g.N / T;
    G.start[p] = total;
    const long tiles = (long)(g.M / T) * (g.N / T);
    // split long K into slices of >= 512 (8 K-tiles): measured on the transformer's
    // dW + dX groups, where the K = d_ff input gradient otherwise runs 4x the
    // K-steps of its neighbour (g_group_split = 0 disables, for A/B runs).  Big
    // tiles split further while the problem has fewer tiles than CUs.
    int sp = 1;
    const int minslice = T >= 128 ? 4 : 8;
    if (g_group_split && ws && counters)
      while (sp < 8 && (g.K / (2 * sp)) % DMA_BK == 0 && g.K / (2 * sp) >= minslice * DMA_BK &&
             (T < 128 || tiles * sp < 256))
        sp *= 2;
    if (sp > 1 && (wsused + tiles * sp * T * T > ws_floats || cntused + tiles > n_counters)) sp = 1;
    G.splits[p] = sp;
    G.wsoff[p] = wsused;
    G.cntoff[p] = (int)cntused;
    G.vec[p] = g_epi_vec && T * T >= 2048 && (long)g.M * g.N >= g_epi_vec_min && epi_vec_ok(g, 1);
    if (sp > 1) { wsused += tiles * sp * T * T; cntused += tiles; }
    total += (int)(tiles * sp);
  }
  G.start[n] = total;
  return total;
}

template <int TMN>
static void group_launch(const GemmGroup& G, int total, bool tail, hipStream_t st) {
  if (tail)  // only then pay for the tail checks in the K loop (measured ~5 % on the transformer's groups)
    hipLaunchKernelGGL((gemm_dma_group_kernel<3, true, TMN, TMN>), dim3(total), dim3(256), 0, st, G);
  else
    hipLaunchKernelGGL((gemm_dma_group_kernel<3, false, TMN, TMN>), dim3(total), dim3(256), 0, st, G);
}

// groups of at least this many FLOPs launch problem by problem (JDT_GEMM_GROUP_FLOPS)
static long g_group_max_flops = -1;
static long group_max_flops() {
  if (g_group_max_flops < 0) {
    const char* e = getenv("JDT_GEMM_GROUP_FLOPS");
    g_group_max_flops = e ? atol(e) : (1L << 30);
  }
  return g_group_max_flops;
}

static int gemm_dma_group(const GemmArgs* gs, int n, float* ws, long ws_floats, unsigned* counters, long n_counters,
                          hipStream_t st) {
  if (g_gemm_no_dma || n < 1 || n > GROUP_MAX) return 1;
  long flops = 0;
  bool m64 = true, m128 = true;
  for (int p = 0; p < n; ++p) {
    const GemmArgs& g = gs[p];
    auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
    if (g.a_f32 || g.b_f32 || g.K % 32 || g.K <= 0 || g.M % 32 || g.N % 32 || g.M <= 0 || g.N <= 0 || !al(g.A) ||
        !al(g.B) || g.lda % 8 || g.ldb % 8 || g.zin > 1)
      return 1;
    flops += 2L * g.M * g.N * g.K;
    m64 &= g.M % 64 == 0 && g.N % 64 == 0;
    m128 &= g.M % 128 == 0 && g.N % 128 == 0;
  }
  // Big groups (>= 1 GFLOP, e.g. the 2048-token transformer backward) are launched
  // as separate single-problem launches: measured (tools/bench_gemm.py --groups) the
  // per-problem tile/split heuristic of jdt_gemm beats one shared grid there by
  // 1.3-2.3x (fc2 bwd group 82 us grouped vs 36 us as two launches); the grouped
  // grid pays off for the small microbatch problems (launch gaps dominate).
  int T = g_group_tile;
  if (T == 0 && flops >= group_max_flops()) return 1;
  if (T == 0) T = (m64 && flops >= (1L << 29)) ? 64 : 32;
  if ((T == 128 && !m128) || (T == 64 && !m64)) T = 32;
  GemmGroup G{};
  const int total = T == 128 ? group_plan<128>(gs, n, G, ws, ws_floats, counters, n_counters)
                  : T == 64  ? group_plan<64>(gs, n, G, ws, ws_floats, counters, n_counters)
                             : group_plan<32>(gs, n, G, ws, ws_floats, counters, n_counters);
  if (total <= 0) return 1;
  bool tail = false;
  for (int p = 0; p < n; ++p) tail |= (gs[p].K / G.splits[p]) % DMA_BK != 0;
  if (T == 128) group_launch<4>(G, total, tail, st);
  else if (T == 64) group_launch<2>(G, total, tail, st);
  else group_launch<1>(G, total, tail, st);
  return HIP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------
// LayerNorm fused into the A operand of a GEMM:  C = epilogue( LN(X) . W )
// (pre-LN transformer: LN1 -> QKV projection, LN2 -> fc1, LN_f -> LM head).
// X is [M, K] bf16 with K = 512 * NV (the model width: a whole row is one 16-byte
// load per lane per 512 columns), W the [K, N] ("kn") bf16 weight.  Each workgroup
// normalises its BM rows in a prologue -- one wave per row, fp32 statistics with
// the DPP wave sums and the exact arithmetic of ln_fwd_kernel, so the bf16 values
// are bit-identical to the unfused LayerNorm -- straight into a RESIDENT LDS image
// of the whole BM x K A operand (the swizzled [BM][64] row images dma_frag reads);
// only W streams through the LDS-DMA ring.  The workgroups of the first column
// block also store Y = LN(X) and the row statistics (the backward's weight
// gradient and LayerNorm backward read them), so the LayerNorm launch and its
// activation round trip disappear.  W's first ring slots are issued before the
// prologue, so their landing overlaps the row loads.
struct LnArgs {
  const bf16_t* X; long ldx;
  const float* gamma; const float* beta; float eps;
  bf16_t* Y; long ldy;          // LN(X) (bf16), written by column block 0
  float* mean; float* rstd;     // per-row statistics (fp32), column block 0
};

template <int WM, int WN, int TM, int TN, int NV>
__global__ void __launch_bounds__(64 * WM * WN) gemm_ln_kernel(GemmArgs g, LnArgs L, int tiles_n, int vec) {
  constexpr int NW = WM * WN;
  constexpr int BM = WM * TM * 16, BN = WN * TN * 16, BK = DMA_BK, KD = 512 * NV, NKT = KD / BK;
  constexpr int S = 3;                       // W ring slots
  constexpr int AIMG = BM * KD;              // resident A image (bf16)
  constexpr int BSTAGE = BN * BK;
  constexpr int LPW = BN / (8 * NW);         // W glds per wave per slot
  static_assert(LPW >= 1 && (S - 2) * LPW <= 63, "ring");
  static_assert((BM * (BN + 4) + 4) * 4 <= (AIMG + S * BSTAGE) * 2, "output image fits");
  __shared__ __attribute__((aligned(16))) bf16_t smem[AIMG + S * BSTAGE];
  const int nwg = gridDim.x;
  int bid = blockIdx.x;
  {
    const int xcd = bid % 8, q = nwg / 8, rr = nwg % 8;
    bid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
  }
  const int tmi = bid / tiles_n, tni = bid % tiles_n;
  const int tm0 = tmi * BM, tn0 = tni * BN;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const bf16_t* Bb = static_cast<const bf16_t*>(g.B) + tn0;  // [K][N]: k-row image
  bf16_t* ring = smem + AIMG;
  auto issue = [&](int kt) { stage_op<BN, true, NW>(Bb, g.ldb, kt * BK, ring + (kt % S) * BSTAGE, wid, lane); };
#pragma unroll
  for (int s = 0; s < S - 1; ++s) issue(s);

  // ---- LN prologue: wave wid normalises rows wid, wid + NW, ...
  float4 ga[NV][2], be[NV][2];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int col = (v * 64 + lane) * 8;
    ga[v][0] = *reinterpret_cast<const float4*>(L.gamma + col);
    ga[v][1] = *reinterpret_cast<const float4*>(L.gamma + col + 4);
    be[v][0] = *reinterpret_cast<const float4*>(L.beta + col);
    be[v][1] = *reinterpret_cast<const float4*>(L.beta + col + 4);
  }
  const bool writer = tni == 0;
  // every row load of this wave in flight at once (a load -> reduce -> store loop
  // would pay one dependent memory round trip per row)
  constexpr int RPW = BM / NW;
  u32x4 rows_in[RPW][NV];
#pragma unroll
  for (int i = 0; i < RPW; ++i)
#pragma unroll
    for (int v = 0; v < NV; ++v)
      rows_in[i][v] = *reinterpret_cast<const u32x4*>(L.X + (long)(tm0 + wid + i * NW) * L.ldx + (v * 64 + lane) * 8);
#pragma unroll
  for (int i = 0; i < RPW; ++i) {
    const int r = wid + i * NW, row = tm0 + r;
    const u32x4* p = rows_in[i];
    float x[NV][8];
    float sum = 0.f;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x[v][2 * j] = bf2f((bf16_t)(p[v][j] & 0xffff));
        x[v][2 * j + 1] = bf2f((bf16_t)(p[v][j] >> 16));
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) sum += x[v][j];
    }
    const float mean = __fdiv_rn(wave_sum_dpp(sum), (float)KD);   // same arithmetic as ln_fwd_kernel
    float q = 0.f;
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
      for (int j = 0; j < 8; ++j) q = ln_sq_acc(q, x[v][j], mean);
    const float rstd = rsqrtf(__fadd_rn(__fdiv_rn(wave_sum_dpp(q), (float)KD), L.eps));
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const float gg[8] = {ga[v][0].x, ga[v][0].y, ga[v][0].z, ga[v][0].w, ga[v][1].x, ga[v][1].y, ga[v][1].z, ga[v][1].w};
      const float bb[8] = {be[v][0].x, be[v][0].y, be[v][0].z, be[v][0].w, be[v][1].x, be[v][1].y, be[v][1].z, be[v][1].w};
      u32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float a = ln_norm(x[v][2 * j], mean, rstd, gg[2 * j], bb[2 * j]);
        const float b = ln_norm(x[v][2 * j + 1], mean, rstd, gg[2 * j + 1], bb[2 * j + 1]);
        o[j] = (unsigned)f2bf(a) | ((unsigned)f2bf(b) << 16);
      }
      // column block (v * 64 + lane) * 8 -> K sub-tile kt = v * 8 + lane / 8, chunk lane % 8
      const int kt = v * 8 + (lane >> 3), c = lane & 7;
      *reinterpret_cast<u32x4*>(smem + kt * (BM * BK) + r * BK + ((c ^ (r & 7)) << 3)) = o;
      if (writer) *reinterpret_cast<u32x4*>(L.Y + (long)row * L.ldy + (v * 64 + lane) * 8) = o;
    }
    if (writer && lane == 0) {
      L.mean[row] = mean;
      L.rstd[row] = rstd;
    }
  }

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int kt = 0; kt < NKT; ++kt) {
    // W slot kt landed (counted vmcnt) and, on the first pass, every wave's A-image
    // writes are done (the wait's lgkmcnt(0) + barrier)
    dma_wait_barrier<LPW, S - 2>(min(S - 2, NKT - 1 - kt));
    if (kt + S - 1 < NKT) issue(kt + S - 1);
    const bf16_t* As = smem + kt * (BM * BK);
    const bf16_t* Bs = ring + (kt % S) * BSTAGE;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = frag_op<BM>(As, false, (wm * TM + i) * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = frag_op<BN>(Bs, true, (wn * TN + j) * 16, kk, lane);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(af[i]));
#pragma unroll
      for (int j = 0; j < TN; ++j) asm volatile("" : "+v"(bfr[j]));
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16x16x32(af[i], bfr[j], acc[i][j]);
    }
  }
  __syncthreads();
  if (vec)
    gemm_finish_vec<BM, BN, TM, TN, 64 * NW>(g, acc, tm0, tn0, 0, wm, wn, lane, tid, 1, 0, 0, nullptr, nullptr,
                                             reinterpret_cast<float*>(smem));
  else if constexpr (NW == 4)
    gemm_finish<BM, BN, TM, TN>(g, acc, tm0, tn0, 0, wid, wm, wn, lane, tid, 1, 0, 0, nullptr, nullptr,
                                reinterpret_cast<int*>(smem));
}

template <int WM, int WN, int TM, int TN, int NV>
static int launch_ln(const GemmArgs& g, const LnArgs& L, hipStream_t st) {
  constexpr int BM = WM * TM * 16, BN = WN * TN * 16;
  if (g.M % BM || g.N % BN) return -2;
  const int tiles_n = g.N / BN;
  const int vec = epi_vec_ok(g, 1);
  hipLaunchKernelGGL((gemm_ln_kernel<WM, WN, TM, TN, NV>), dim3((g.M / BM) * tiles_n), dim3(64 * WM * WN), 0, st, g, L,
                     tiles_n, vec);
  return HIP_LAUNCH_CHECK();
}
}  // namespace jdt

using namespace jdt;

// Tile choice: the tutorial GEMMs are small (M = 4..128 rows per device), so the
// heuristic favours enough workgroups to cover the chip over per-tile reuse.
JDT_API void jdt_gemm_set_preload(int on) { g_gemm_no_preload = !on; }
JDT_API void jdt_gemm_set_exact(int pre) { g_exact_pre = pre; }
JDT_API void jdt_gemm_set_dma(int on) { g_gemm_no_dma = !on; }
JDT_API void jdt_gemm_set_epi_vec(int on) { g_epi_vec = on; }
JDT_API void jdt_gemm_set_epi_vec_min(long n) { g_epi_vec_min = n; }
JDT_API void jdt_gemm_set_r(int r) { g_dma_r = r; }
JDT_API void jdt_gemm_set_tune(int on) { g_gemm_tune = on; }
// write-through stores in the vectorised GEMM epilogue (bit 0: C / Zout, bit 1: AdamW state
// + shadow); a device global read once per epilogue, set before any capture (A/B)
JDT_API int jdt_gemm_set_wt(int mask) {
  return hipMemcpyToSymbol(HIP_SYMBOL(g_gemm_wt_dev), &mask, sizeof(int)) == hipSuccess ? 0 : -1;
}

JDT_API int jdt_gemm(const GemmArgs* ga, int batch, int cfg, int splits, float* ws, long ws_floats,
                     unsigned* counters, long n_counters, void* stream) {
  const GemmArgs& g = *ga;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (g.M <= 0 || g.N <= 0) return 0;
  if (cfg < 0 || cfg >= 10) {
    const int rc = gemm_dma(g, batch, cfg, splits, ws, ws_floats, counters, n_counters, st);
    if (rc != 1) return rc;  // 1 = shape outside the LDS-DMA envelope: register-staged kernels below
    if (cfg >= 10) return -1;
  }
  if (cfg < 0) {
    const long t128 = (long)((g.M + 63) / 64) * ((g.N + 127) / 128) * batch;
    const long t64 = (long)((g.M + 63) / 64) * ((g.N + 63) / 64) * batch;
    const long t32 = (long)((g.M + 31) / 32) * ((g.N + 63) / 64) * batch;
    if (g.M >= 64 && g.N >= 128 && t128 >= 256) cfg = 3;
    else if (g.M >= 64 && t64 >= 96) cfg = 2;
    else if (g.M > 16 && t32 >= 64) cfg = 1;
    else if (g.M <= 16) cfg = 0;
    else cfg = (g.N <= 32) ? 4 : 0;
  }
  switch (cfg) {
    case 0: return launch_cfg<1, 4, 1, 1, 64>(g, batch, splits, ws, ws_floats, counters, n_counters, st);   // 16 x 64
    case 1: return launch_cfg<2, 2, 1, 2, 64>(g, batch, splits, ws, ws_floats, counters, n_counters, st);   // 32 x 64
    case 2: return launch_cfg<2, 2, 2, 2, 32>(g, batch, splits, ws, ws_floats, counters, n_counters, st);   // 64 x 64
    case 3: return launch_cfg<2, 2, 2, 4, 32>(g, batch, splits, ws, ws_floats, counters, n_counters, st);   // 64 x 128
    case 4: return launch_cfg<4, 1, 1, 1, 64>(g, batch, splits, ws, ws_floats, counters, n_counters, st);   // 64 x 16
    default: return -1;
  }
}

JDT_API int jdt_gemm_args_size() { return (int)sizeof(GemmArgs); }
JDT_API int jdt_ln_args_size() { return (int)sizeof(LnArgs); }

// C = epilogue(LN(X) . W) with LN(X) and its row statistics also stored (see
// gemm_ln_kernel).  X [M, K] bf16 (K in {512, 1024}, rows 16-byte aligned), W
// [K, N] bf16 "kn"; M % 32 == 0, N % 64 == 0.  Returns -2 outside that envelope.
static int g_ln_cfg = 0;  // jdt_gemm_ln_set_cfg: force a tile (sweeps); 0 = heuristic
// the fused kernel's tile config for (g, L), or -2: not eligible (LN + GEMM run apart)
static int gemm_ln_cfg(const GemmArgs& g, const LnArgs& L) {
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (g.a_f32 || g.b_f32 || !g.b_trans || g.accumulate || g.Zin || g.zin > 1 || (g.K != 512 && g.K != 1024) ||
      g.M % 32 || g.N % 64 || !al(L.X) || !al(L.Y) || !al(g.B) || L.ldx % 8 || L.ldy % 8 || g.ldb % 8 ||
      !al(L.gamma) || !al(L.beta))
    return -2;
  int cfg = g_ln_cfg;
  if (cfg <= 0) {
    // measured (tools/bench_ln_gemm.py): the fused kernel normalises each row once per
    // column block, so it only pays off while the separate LN launch is a large share:
    // M <= 512 (round 3, 32 x 64 tile: qkv 512 rows 8.39 vs 9.50 us LN + GEMM, fc1
    // 512 rows 9.79 vs 10.12, 256 rows 6.95 vs 7.42; profiles/r3_ln_gemm_sweep.txt);
    // the 2048-row shapes run LN + GEMM (the fused 16 x 64 tile only ties them)
    if (g.M > 512 || g.N > 2048) return -2;
    cfg = 1;
  }
  return g.K == 1024 || cfg <= 4 ? cfg : -2;   // K = 1024 has one config
}

// 1: jdt_gemm_ln would run the fused kernel for (g, L); 0: it would return -2
JDT_API int jdt_gemm_ln_eligible(const GemmArgs* ga, const LnArgs* la) { return gemm_ln_cfg(*ga, *la) > 0; }

JDT_API int jdt_gemm_ln(const GemmArgs* ga, const LnArgs* la, void* stream) {
  const GemmArgs& g = *ga;
  const LnArgs& L = *la;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int cfg = gemm_ln_cfg(g, L);
  if (cfg < 0) return -2;
  if (g.K == 1024) return launch_ln<2, 2, 1, 2, 2>(g, L, st);
  switch (cfg) {
    case 1: return launch_ln<2, 2, 1, 2, 1>(g, L, st);   // 32 x 64
    case 2: return launch_ln<2, 2, 2, 2, 1>(g, L, st);   // 64 x 64
    case 3: return launch_ln<2, 2, 1, 4, 1>(g, L, st);   // 32 x 128
    case 4: return launch_ln<2, 2, 2, 4, 1>(g, L, st);   // 64 x 128
    default: return -2;
  }
}
JDT_API void jdt_gemm_ln_set_cfg(int c) { g_ln_cfg = c; }

// n GEMMs (no batch) in one launch; 1 = not eligible (launch them one by one).
JDT_API int jdt_gemm_group(const GemmArgs* gs, int n, float* ws, long ws_floats, unsigned* counters, long n_counters,
                           void* stream) {
  return gemm_dma_group(gs, n, ws, ws_floats, counters, n_counters, static_cast<hipStream_t>(stream));
}
JDT_API void jdt_gemm_set_group_split(int on) { g_group_split = on; }
JDT_API void jdt_gemm_set_group_m(int gm) { g_group_m = gm; }
JDT_API void jdt_gemm_set_group_tile(int t) { g_group_tile = t; }

// The W pass (gemm_wpass_kernel): plan the prefix table of `n` weight-gradient problems
// into `out` (host memory; the caller copies it to the device once and replays it) for
// tile config `cfg` (0: 64 x 64 of 16x16x32 MFMAs, 1: 64 x 64 of 32x32x16, 2: 128 x 128
// of 32x32x16, 3: 32 x 64, 4: 64 x 128, 5: 128 x 64).  Split-K per problem while the whole launch has fewer than
// two workgroups per CU.  Returns the workgroup count, or < 0 outside the envelope (a
// problem not "km" x "kn" bf16 with 16-byte aligned operands and fp32 output rows, a
// shape not a multiple of the tile, K not a multiple of 64, > WP_MAX problems).
template <int BM, int BN>
static int wpass_plan(const GemmArgs* gs, int n, GemmWTable* out, float* ws, long ws_floats, unsigned* counters,
                      long n_counters) {
  if (n <= 0 || n > WP_MAX) return -2;
  auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  long tiles_all = 0;
  for (int p = 0; p < n; ++p) {
    const GemmArgs& g = gs[p];
    if (!g.a_trans || !g.b_trans || g.a_f32 || g.b_f32 || !g.c_f32 || g.M % BM || g.N % BN || g.K % DMA_BK ||
        !al(g.A) || !al(g.B) || g.lda % 8 || g.ldb % 8 || !epi_vec_ok(g, 1) || g.Zin || g.Zout || g.resid ||
        g.keep_prob < 1.f)
      return -2;
    tiles_all += (long)(g.M / BM) * (g.N / BN);
  }
  int total = 0;
  long wsused = 0, cntused = 0;
  out->n = n;
  out->ws = ws;
  out->counters = counters;
  for (int p = 0; p < n; ++p) {
    const GemmArgs& g = gs[p];
    out->g[p] = g;
    out->tiles_n[p] = g.N / BN;
    out->start[p] = total;
    const long tiles = (long)(g.M / BM) * (g.N / BN);
    int sp = 1;
    while (sp < 8 && tiles_all * sp < 512 && (g.K / (2 * sp)) % DMA_BK == 0 && g.K / (2 * sp) >= 8 * DMA_BK) sp *= 2;
    if (sp > 1 && (!ws || !counters || wsused + tiles * sp * BM * BN > ws_floats || cntused + tiles > n_counters))
      sp = 1;
    out->splits[p] = sp;
    out->wsoff[p] = wsused;
    out->cntoff[p] = (int)cntused;
    if (sp > 1) { wsused += tiles * sp * BM * BN; cntused += tiles; }
    total += (int)(tiles * sp);
  }
  out->start[n] = total;
  out->total = total;
  return total;
}

JDT_API int jdt_gemm_wpass_table_bytes() { return (int)sizeof(GemmWTable); }
JDT_API int jdt_gemm_wpass_plan(const GemmArgs* gs, int n, int cfg, void* out, float* ws, long ws_floats,
                                unsigned* counters, long n_counters) {
  GemmWTable* t = static_cast<GemmWTable*>(out);
  switch (cfg) {
    case 0: case 1: return wpass_plan<64, 64>(gs, n, t, ws, ws_floats, counters, n_counters);
    case 2: return wpass_plan<128, 128>(gs, n, t, ws, ws_floats, counters, n_counters);
    case 3: return wpass_plan<32, 64>(gs, n, t, ws, ws_floats, counters, n_counters);
    case 4: return wpass_plan<64, 128>(gs, n, t, ws, ws_floats, counters, n_counters);
    case 5: return wpass_plan<128, 64>(gs, n, t, ws, ws_floats, counters, n_counters);
    default: return -2;
  }
}
// launch the planned table (device copy) with `total` workgroups
JDT_API int jdt_gemm_wpass_launch(const void* table_dev, int total, int cfg, void* stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  const GemmWTable* t = static_cast<const GemmWTable*>(table_dev);
  if (total <= 0) return 0;
  switch (cfg) {
    case 0: hipLaunchKernelGGL((gemm_wpass_kernel<2, 2, 16, 3>), dim3(total), dim3(256), 0, st, t); break;
    case 1: hipLaunchKernelGGL((gemm_wpass_kernel<1, 1, 32, 3>), dim3(total), dim3(256), 0, st, t); break;
    case 2: hipLaunchKernelGGL((gemm_wpass_kernel<2, 2, 32, 3>), dim3(total), dim3(256), 0, st, t); break;
    case 3: hipLaunchKernelGGL((gemm_wpass_kernel<1, 2, 16, 3>), dim3(total), dim3(256), 0, st, t); break;
    // 2 workgroups per CU (74 KB of LDS each): one's AdamW epilogue under the other's main loop
    case 4: hipLaunchKernelGGL((gemm_wpass_kernel<1, 2, 32, 3>), dim3(total), dim3(256), 0, st, t); break;
    case 5: hipLaunchKernelGGL((gemm_wpass_kernel<2, 1, 32, 3>), dim3(total), dim3(256), 0, st, t); break;
    default: return -2;
  }
  return HIP_LAUNCH_CHECK();
}
