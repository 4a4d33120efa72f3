// Fused (flash-style) causal self-attention for the transformer tutorial model,
// head dim 64, bf16 in/out, fp32 softmax statistics.  q/k/v are read in place
// from the fused [B*S, 3*H*64] QKV projection; O is written in place into the
// [B*S, H*64] attention output; nothing of size S x S ever reaches HBM.
//
// forward  grid (S/64 query blocks, B*H); 4 waves x 16 query rows.
//   Per 64-key tile: K (row-major) and V (transposed) staged in LDS,
//   S = Q K^T on MFMA (Q fragments in registers), online softmax in registers
//   (row stats reduced over the 16 lanes that share a row), P -> per-wave LDS
//   tile (bf16) -> O += P V on MFMA.  Saves LSE (of the scaled scores) per row.
// backward  ONE launch, grid (S/64 key blocks, B*H), each wave owns 16 keys:
//   per 64-query tile delta = rowsum(dO * O) (recomputed, cheaper than a launch),
//   P^T = exp(scale K Q^T - LSE), dP^T = V dO^T, dS^T = P^T (dP^T - delta),
//   dV += P^T dO, dK += dS^T Q (fp32 accumulators in registers for the whole
//   sweep), dQ += dS K summed across key blocks with fp32 atomics into a
//   persistent zeroed workspace; the key block that arrives last for its
//   (batch, head) (ticket) converts that head's dQ to bf16 into the QKV
//   gradient and re-zeroes the workspace -- no memset, delta or convert launch.
#include "common.h"

namespace jdt {

constexpr int FD = 64;          // head dim
constexpr int FB = 64;          // query / key tile
constexpr int FLD = FB + 8;     // padded LDS row (bf16 elements)

__device__ __forceinline__ bf16x8 ld8(const bf16_t* p) { return *reinterpret_cast<const bf16x8*>(p); }

// stage a [64 rows][64 cols] bf16 tile (global row stride ld) into LDS, row-major
// and/or transposed; rows >= nrows are zero.
__device__ __forceinline__ void stage_tile(const bf16_t* g, long ld, int nrows, bf16_t* row_major,
                                           bf16_t* transposed) {
  for (int c = threadIdx.x; c < FB * FD / 8; c += 256) {
    const int r = c >> 3, dc = (c & 7) * 8;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (r < nrows) v = *reinterpret_cast<const u32x4*>(g + (long)r * ld + dc);
    if (row_major) *reinterpret_cast<u32x4*>(row_major + r * FLD + dc) = v;
    if (transposed) {
      const unsigned q[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        transposed[(dc + 2 * j) * FLD + r] = (bf16_t)(q[j] & 0xffff);
        transposed[(dc + 2 * j + 1) * FLD + r] = (bf16_t)(q[j] >> 16);
      }
    }
  }
}

__global__ void __launch_bounds__(256) flash_fwd_kernel(const bf16_t* __restrict__ qkv, bf16_t* __restrict__ out,
                                                        float* __restrict__ lse, int S, int H, float scale,
                                                        int causal) {
  __shared__ __attribute__((aligned(16))) bf16_t Ks[FB * FLD];
  __shared__ __attribute__((aligned(16))) bf16_t Vt[FD * FLD];
  __shared__ __attribute__((aligned(16))) bf16_t Ps[4][16 * FLD];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const int d = H * FD, ld3 = 3 * d;
  const int q0 = blockIdx.x * FB, qw = q0 + w * 16;
  const bf16_t* base = qkv + (long)b * S * ld3;

  bf16x8 qf[2];
  {
    const int row = qw + (lane & 15);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      qf[ks] = row < S ? ld8(base + (long)row * ld3 + h * FD + ks * 32 + 8 * (lane >> 4))
                       : (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
  }
  float m[4], l[4];
  f32x4 o[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) { m[e] = -INFINITY; l[e] = 0.f; }
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) o[nt] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int kend = causal ? min(S, q0 + FB) : S;
  for (int k0 = 0; k0 < kend; k0 += FB) {
    __syncthreads();
    stage_tile(base + (long)k0 * ld3 + d + h * FD, ld3, S - k0, Ks, nullptr);
    stage_tile(base + (long)k0 * ld3 + 2 * d + h * FD, ld3, S - k0, nullptr, Vt);
    __syncthreads();
    // S = Q K^T (16 x 64 per wave)
    f32x4 s[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      s[nt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        s[nt] = mfma16x16x32(qf[ks], ld8(&Ks[(nt * 16 + (lane & 15)) * FLD + ks * 32 + 8 * (lane >> 4)]), s[nt]);
    }
    // online softmax over this tile (row r = (lane>>4)*4 + e; key column nt*16 + (lane&15))
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int qrow = qw + (lane >> 4) * 4 + e;
      float mx = -INFINITY;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int key = k0 + nt * 16 + (lane & 15);
        float v = s[nt][e] * scale;
        if (key >= S || (causal && key > qrow)) v = -INFINITY;
        s[nt][e] = v;
        mx = fmaxf(mx, v);
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
      const float mnew = fmaxf(m[e], mx);
      const float alpha = (mnew == -INFINITY) ? 1.f : __expf(m[e] - mnew);
      float rs = 0.f;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const float p = (mnew == -INFINITY) ? 0.f : __expf(s[nt][e] - mnew);
        s[nt][e] = p;
        rs += p;
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) rs += __shfl_xor(rs, off, 64);
      l[e] = l[e] * alpha + rs;
      m[e] = mnew;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) o[nt][e] *= alpha;
    }
    // P (bf16) -> per-wave LDS tile [row][key] so it can be the A operand of P V
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int e = 0; e < 4; ++e) Ps[w][((lane >> 4) * 4 + e) * FLD + nt * 16 + (lane & 15)] = f2bf(s[nt][e]);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's P writes land before its reads
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 pa = ld8(&Ps[w][(lane & 15) * FLD + ks * 32 + 8 * (lane >> 4)]);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        o[nt] = mfma16x16x32(pa, ld8(&Vt[(nt * 16 + (lane & 15)) * FLD + ks * 32 + 8 * (lane >> 4)]), o[nt]);
    }
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int row = qw + (lane >> 4) * 4 + e;
    if (row >= S) continue;
    const float inv = 1.f / l[e];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
      out[((long)b * S + row) * d + h * FD + nt * 16 + (lane & 15)] = f2bf(o[nt][e] * inv);
    if ((lane & 15) == 0) lse[(long)bh * S + row] = m[e] + __logf(l[e]);
  }
}

__global__ void __launch_bounds__(256) flash_bwd_kernel(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ o,
                                                        const bf16_t* __restrict__ dout, const float* __restrict__ lse,
                                                        bf16_t* __restrict__ dqkv, float* __restrict__ dq_acc,
                                                        unsigned* __restrict__ tickets, float* __restrict__ dbias,
                                                        int S, int H, float scale, int causal) {
  __shared__ __attribute__((aligned(16))) bf16_t Qs[FB * FLD];
  __shared__ __attribute__((aligned(16))) bf16_t Qt[FD * FLD];
  __shared__ __attribute__((aligned(16))) bf16_t dOs[FB * FLD];
  __shared__ __attribute__((aligned(16))) bf16_t dOt[FD * FLD];
  __shared__ __attribute__((aligned(16))) bf16_t Kt[FD * FLD];
  __shared__ __attribute__((aligned(16))) bf16_t Pw[4][16 * FLD];
  __shared__ __attribute__((aligned(16))) bf16_t dSw[4][16 * FLD];
  __shared__ __attribute__((aligned(16))) bf16_t dSq[FB * FLD];   // dS[q][key] for dQ
  __shared__ float lse_s[FB], delta_s[FB];
  __shared__ int last_s;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int bh = blockIdx.y, b = bh / H, h = bh % H;
  const int d = H * FD, ld3 = 3 * d;
  const int k0 = blockIdx.x * FB, kw = k0 + w * 16;
  const bf16_t* base = qkv + (long)b * S * ld3;
  const bf16_t* dbase = dout + (long)b * S * d;

  bf16x8 kf[2], vf[2];
  {
    const int key = kw + (lane & 15);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = ks * 32 + 8 * (lane >> 4);
      kf[ks] = key < S ? ld8(base + (long)key * ld3 + d + h * FD + c) : (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
      vf[ks] = key < S ? ld8(base + (long)key * ld3 + 2 * d + h * FD + c) : (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  stage_tile(base + (long)k0 * ld3 + d + h * FD, ld3, S - k0, nullptr, Kt);
  f32x4 dk[4], dv[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) { dk[nt] = (f32x4){0.f, 0.f, 0.f, 0.f}; dv[nt] = dk[nt]; }

  for (int q0 = causal ? k0 : 0; q0 < S; q0 += FB) {
    __syncthreads();
    stage_tile(base + (long)q0 * ld3 + h * FD, ld3, S - q0, Qs, Qt);
    stage_tile(dbase + (long)q0 * d + h * FD, d, S - q0, dOs, dOt);
    if (threadIdx.x < FB) {
      // delta[q] = dO[q, h, :] . O[q, h, :]
      const int q = q0 + threadIdx.x;
      float dl = 0.f;
      if (q < S) {
        const long off = ((long)b * S + q) * d + h * FD;
#pragma unroll
        for (int c = 0; c < FD; c += 8) {
          const u32x4 x = *reinterpret_cast<const u32x4*>(dout + off + c);
          const u32x4 y = *reinterpret_cast<const u32x4*>(o + off + c);
          const unsigned wx[4] = {x.x, x.y, x.z, x.w}, wy[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
          for (int j = 0; j < 4; ++j)
            dl += bf2f((bf16_t)(wx[j] & 0xffff)) * bf2f((bf16_t)(wy[j] & 0xffff)) +
                  bf2f((bf16_t)(wx[j] >> 16)) * bf2f((bf16_t)(wy[j] >> 16));
        }
      }
      lse_s[threadIdx.x] = q < S ? lse[(long)bh * S + q] : 0.f;
      delta_s[threadIdx.x] = dl;
    }
    __syncthreads();
    // S^T = K Q^T, dP^T = V dO^T   (rows: this wave's 16 keys; cols: 64 queries)
    f32x4 st[4], dpt[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      st[nt] = (f32x4){0.f, 0.f, 0.f, 0.f};
      dpt[nt] = st[nt];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int c = (nt * 16 + (lane & 15)) * FLD + ks * 32 + 8 * (lane >> 4);
        st[nt] = mfma16x16x32(kf[ks], ld8(&Qs[c]), st[nt]);
        dpt[nt] = mfma16x16x32(vf[ks], ld8(&dOs[c]), dpt[nt]);
      }
    }
    // P^T, dS^T (bf16) -> per-wave LDS [key][q]; dS -> shared [q][key]
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int ql = nt * 16 + (lane & 15), q = q0 + ql;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int kl = (lane >> 4) * 4 + e, key = kw + kl;
        const bool ok = q < S && key < S && !(causal && key > q);
        const float p = ok ? __expf(st[nt][e] * scale - lse_s[ql]) : 0.f;
        const float ds = p * (dpt[nt][e] - delta_s[ql]);
        Pw[w][kl * FLD + ql] = f2bf(p);
        const bf16_t dsb = f2bf(ds);
        dSw[w][kl * FLD + ql] = dsb;
        dSq[ql * FLD + w * 16 + kl] = dsb;
      }
    }
    __syncthreads();
    // dV += P^T dO ; dK += dS^T Q   (K-dim = the 64 queries)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ca = (lane & 15) * FLD + ks * 32 + 8 * (lane >> 4);
      const bf16x8 pa = ld8(&Pw[w][ca]), sa = ld8(&dSw[w][ca]);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int cb = (nt * 16 + (lane & 15)) * FLD + ks * 32 + 8 * (lane >> 4);
        dv[nt] = mfma16x16x32(pa, ld8(&dOt[cb]), dv[nt]);
        dk[nt] = mfma16x16x32(sa, ld8(&Qt[cb]), dk[nt]);
      }
    }
    // dQ[q0 + w*16 .. +16][:] += dS K  (K-dim = this block's 64 keys), fp32 atomics across key blocks
    f32x4 dq[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) dq[nt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const bf16x8 sa = ld8(&dSq[(w * 16 + (lane & 15)) * FLD + ks * 32 + 8 * (lane >> 4)]);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        dq[nt] = mfma16x16x32(sa, ld8(&Kt[(nt * 16 + (lane & 15)) * FLD + ks * 32 + 8 * (lane >> 4)]), dq[nt]);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int q = q0 + w * 16 + (lane >> 4) * 4 + e;
      if (q >= S) continue;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        atomicAdd(dq_acc + ((long)b * S + q) * d + h * FD + nt * 16 + (lane & 15), dq[nt][e] * scale);
    }
  }
  // dK, dV -> the K and V column blocks of dQKV; with dbias, their column sums
  // (the k/v bias gradient, over exactly the stored bf16 values) go out with one
  // atomic per column per wave
  float sk[4] = {0.f, 0.f, 0.f, 0.f}, sv[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int key = kw + (lane >> 4) * 4 + e;
    if (key >= S) continue;
    bf16_t* row = dqkv + ((long)b * S + key) * ld3 + h * FD + (lane & 15);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const bf16_t kb = f2bf(dk[nt][e] * scale), vb = f2bf(dv[nt][e]);
      row[d + nt * 16] = kb;
      row[2 * d + nt * 16] = vb;
      sk[nt] += bf2f(kb);
      sv[nt] += bf2f(vb);
    }
  }
  if (dbias) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      sk[nt] += __shfl_xor(sk[nt], 16, 64);
      sk[nt] += __shfl_xor(sk[nt], 32, 64);
      sv[nt] += __shfl_xor(sv[nt], 16, 64);
      sv[nt] += __shfl_xor(sv[nt], 32, 64);
    }
    if (lane < 16) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        atomicAdd(dbias + d + h * FD + nt * 16 + lane, sk[nt]);
        atomicAdd(dbias + 2 * d + h * FD + nt * 16 + lane, sv[nt]);
      }
    }
  }
  // last key block of this (batch, head): dQ fp32 -> bf16, workspace re-zeroed.
  // The dQ atomics are device-scope (performed past the per-XCD L2s); drain
  // them (vmcnt) before the ticket; the last arriver acquires at agent scope
  // (invalidating its XCD's L2) and then reads the head's dQ with plain
  // 16-byte loads, all in flight at once.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(tickets + bh, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == gridDim.x - 1;
    if (last) __hip_atomic_store(tickets + bh, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last_s = last;
  }
  __syncthreads();
  if (!last_s) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  constexpr int QV = FD / 4;  // float4 per row; thread t always owns columns 4 (t % QV) .. +3
  float sq[4] = {0.f, 0.f, 0.f, 0.f};
  for (int i0 = 0; i0 < S * QV; i0 += 256 * 8) {
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * 256 + threadIdx.x;
      v[u] = i < S * QV ? *reinterpret_cast<const float4*>(dq_acc + ((long)b * S + i / QV) * d + h * FD + (i % QV) * 4)
                        : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * 256 + threadIdx.x;
      if (i >= S * QV) continue;
      const int q = i / QV, c = (i % QV) * 4;
      *reinterpret_cast<float4*>(dq_acc + ((long)b * S + q) * d + h * FD + c) = make_float4(0.f, 0.f, 0.f, 0.f);
      const bf16_t h0 = f2bf(v[u].x), h1 = f2bf(v[u].y), h2 = f2bf(v[u].z), h3 = f2bf(v[u].w);
      uint2 pk;
      pk.x = (unsigned)h0 | ((unsigned)h1 << 16);
      pk.y = (unsigned)h2 | ((unsigned)h3 << 16);
      *reinterpret_cast<uint2*>(dqkv + ((long)b * S + q) * ld3 + h * FD + c) = pk;
      sq[0] += bf2f(h0); sq[1] += bf2f(h1); sq[2] += bf2f(h2); sq[3] += bf2f(h3);
    }
  }
  if (dbias) {  // q bias gradient: lanes t, t+16, t+32, t+48 of a wave share columns
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      sq[j] += __shfl_xor(sq[j], 16, 64);
      sq[j] += __shfl_xor(sq[j], 32, 64);
    }
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < 4; ++j) atomicAdd(dbias + h * FD + lane * 4 + j, sq[j]);
    }
  }
}

// ---------------------------------------------------------------------------
// Whole-head backward (S <= 128, the tutorial LM's sequence length): ONE
// workgroup of 8 waves per (batch, head), wave w owns keys 16w .. 16w + 15.
// The key-block kernel above splits a head over S/64 workgroups, so dQ (a sum
// over key blocks) needs fp32 atomics into a workspace and a last-arriver
// conversion pass; at S = 128 that atomic / ticket tail and the half-empty
// causal blocks dominated (35 us per launch, 19 TFLOP/s, rocprofv3
// profiles/r2_transformer_merged_tuned_kernel_stats.csv).  Here every key of the
// head is in the workgroup, so per 64-query tile dQ = dS K is one more MFMA
// pass over the shared dS image, written straight to dQKV as bf16: no atomics,
// no workspace, no ticket, and a fixed summation order (deterministic).
constexpr int FS = 128;          // keys per head handled by one workgroup
constexpr int KLD = FS + 8;      // padded [64][128] image row (bf16)

// [64 rows][64 cols] bf16 tile -> LDS (row-major and/or transposed with row
// stride tld), rows >= nrows zero; 512 threads.
__device__ __forceinline__ void stage_tile512(const bf16_t* g, long ld, int nrows, bf16_t* row_major,
                                              bf16_t* transposed, int tld) {
  const int c = threadIdx.x;  // FB * FD / 8 == 512 chunks: one per thread
  const int r = c >> 3, dc = (c & 7) * 8;
  u32x4 v = {0u, 0u, 0u, 0u};
  if (r < nrows) v = *reinterpret_cast<const u32x4*>(g + (long)r * ld + dc);
  if (row_major) *reinterpret_cast<u32x4*>(row_major + r * FLD + dc) = v;
  if (transposed) {
    const unsigned q[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      transposed[(dc + 2 * j) * tld + r] = (bf16_t)(q[j] & 0xffff);
      transposed[(dc + 2 * j + 1) * tld + r] = (bf16_t)(q[j] >> 16);
    }
  }
}

__global__ void __launch_bounds__(512) flash_bwd_head_kernel(const bf16_t* __restrict__ qkv,
                                                             const bf16_t* __restrict__ o,
                                                             const bf16_t* __restrict__ dout,
                                                             const float* __restrict__ lse, bf16_t* __restrict__ dqkv,
                                                             float* __restrict__ dbias, int S, int H, float scale,
                                                             int causal) {
  __shared__ __attribute__((aligned(16))) bf16_t Qs[FB * FLD];
  __shared__ __attribute__((aligned(16))) bf16_t Qt[FD * FLD];
  __shared__ __attribute__((aligned(16))) bf16_t dOs[FB * FLD];
  __shared__ __attribute__((aligned(16))) bf16_t dOt[FD * FLD];
  __shared__ __attribute__((aligned(16))) bf16_t Kt[FD * KLD];     // K^T [dim][key]
  __shared__ __attribute__((aligned(16))) bf16_t Pw[8][16 * FLD];
  __shared__ __attribute__((aligned(16))) bf16_t dSw[8][16 * FLD];
  __shared__ __attribute__((aligned(16))) bf16_t dSq[FB * KLD];    // dS[q][key]
  __shared__ float lse_s[FB], delta_s[FB];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int bh = blockIdx.x, b = bh / H, h = bh % H;
  const int d = H * FD, ld3 = 3 * d;
  const int kw = w * 16;
  const bf16_t* base = qkv + (long)b * S * ld3;
  const bf16_t* dbase = dout + (long)b * S * d;

  bf16x8 kf[2], vf[2];
  {
    const int key = kw + (lane & 15);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int c = ks * 32 + 8 * (lane >> 4);
      kf[ks] = key < S ? ld8(base + (long)key * ld3 + d + h * FD + c) : (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
      vf[ks] = key < S ? ld8(base + (long)key * ld3 + 2 * d + h * FD + c) : (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  stage_tile512(base + d + h * FD, ld3, S, nullptr, Kt, KLD);
  stage_tile512(base + (long)FB * ld3 + d + h * FD, ld3, S - FB, nullptr, Kt + FB, KLD);
  f32x4 dk[4], dv[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) { dk[nt] = (f32x4){0.f, 0.f, 0.f, 0.f}; dv[nt] = dk[nt]; }
  // dQ role of this wave: 16 query rows (w & 3) x 32 dims (w >> 2) of each tile
  const int qr = (w & 3) * 16, nt0 = (w >> 2) * 2;
  float sq[2] = {0.f, 0.f};

  for (int q0 = 0; q0 < S; q0 += FB) {
    __syncthreads();
    stage_tile512(base + (long)q0 * ld3 + h * FD, ld3, S - q0, Qs, Qt, FLD);
    stage_tile512(dbase + (long)q0 * d + h * FD, d, S - q0, dOs, dOt, FLD);
    if (threadIdx.x < FB) {
      const int q = q0 + threadIdx.x;
      float dl = 0.f;
      if (q < S) {
        const long off = ((long)b * S + q) * d + h * FD;
#pragma unroll
        for (int c = 0; c < FD; c += 8) {
          const u32x4 x = *reinterpret_cast<const u32x4*>(dout + off + c);
          const u32x4 y = *reinterpret_cast<const u32x4*>(o + off + c);
          const unsigned wx[4] = {x.x, x.y, x.z, x.w}, wy[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
          for (int j = 0; j < 4; ++j)
            dl += bf2f((bf16_t)(wx[j] & 0xffff)) * bf2f((bf16_t)(wy[j] & 0xffff)) +
                  bf2f((bf16_t)(wx[j] >> 16)) * bf2f((bf16_t)(wy[j] >> 16));
        }
      }
      lse_s[threadIdx.x] = q < S ? lse[(long)bh * S + q] : 0.f;
      delta_s[threadIdx.x] = dl;
    }
    __syncthreads();
    // this wave's keys see any query of the tile (uniform per wave)
    const bool active = kw < S && !(causal && kw > q0 + FB - 1);
    if (active) {
      f32x4 st[4], dpt[4];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        st[nt] = (f32x4){0.f, 0.f, 0.f, 0.f};
        dpt[nt] = st[nt];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const int c = (nt * 16 + (lane & 15)) * FLD + ks * 32 + 8 * (lane >> 4);
          st[nt] = mfma16x16x32(kf[ks], ld8(&Qs[c]), st[nt]);
          dpt[nt] = mfma16x16x32(vf[ks], ld8(&dOs[c]), dpt[nt]);
        }
      }
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const int ql = nt * 16 + (lane & 15), q = q0 + ql;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int kl = (lane >> 4) * 4 + e, key = kw + kl;
          const bool ok = q < S && key < S && !(causal && key > q);
          const float p = ok ? __expf(st[nt][e] * scale - lse_s[ql]) : 0.f;
          const float ds = p * (dpt[nt][e] - delta_s[ql]);
          Pw[w][kl * FLD + ql] = f2bf(p);
          const bf16_t dsb = f2bf(ds);
          dSw[w][kl * FLD + ql] = dsb;
          dSq[ql * KLD + kw + kl] = dsb;
        }
      }
    } else {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int e = 0; e < 4; ++e) dSq[(nt * 16 + (lane & 15)) * KLD + kw + (lane >> 4) * 4 + e] = 0;
    }
    __syncthreads();
    if (active) {
      // dV += P^T dO ; dK += dS^T Q   (K-dim = the 64 queries)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int ca = (lane & 15) * FLD + ks * 32 + 8 * (lane >> 4);
        const bf16x8 pa = ld8(&Pw[w][ca]), sa = ld8(&dSw[w][ca]);
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          const int cb = (nt * 16 + (lane & 15)) * FLD + ks * 32 + 8 * (lane >> 4);
          dv[nt] = mfma16x16x32(pa, ld8(&dOt[cb]), dv[nt]);
          dk[nt] = mfma16x16x32(sa, ld8(&Qt[cb]), dk[nt]);
        }
      }
    }
    // dQ[q0 + qr .. +16][32 dims] = scale * dS K over every key that can be unmasked
    const int kmax = causal ? min(S, q0 + FB) : S;
    f32x4 dq[2];
    dq[0] = (f32x4){0.f, 0.f, 0.f, 0.f};
    dq[1] = dq[0];
    for (int ks = 0; ks < (kmax + 31) / 32; ++ks) {
      const bf16x8 sa = ld8(&dSq[(qr + (lane & 15)) * KLD + ks * 32 + 8 * (lane >> 4)]);
#pragma unroll
      for (int j = 0; j < 2; ++j)
        dq[j] = mfma16x16x32(sa, ld8(&Kt[((nt0 + j) * 16 + (lane & 15)) * KLD + ks * 32 + 8 * (lane >> 4)]), dq[j]);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int q = q0 + qr + (lane >> 4) * 4 + e;
      if (q >= S) continue;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const bf16_t qb = f2bf(dq[j][e] * scale);
        dqkv[((long)b * S + q) * ld3 + h * FD + (nt0 + j) * 16 + (lane & 15)] = qb;
        sq[j] += bf2f(qb);
      }
    }
  }
  float sk[4] = {0.f, 0.f, 0.f, 0.f}, sv[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int key = kw + (lane >> 4) * 4 + e;
    if (key >= S) continue;
    bf16_t* row = dqkv + ((long)b * S + key) * ld3 + h * FD + (lane & 15);
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const bf16_t kb = f2bf(dk[nt][e] * scale), vb = f2bf(dv[nt][e]);
      row[d + nt * 16] = kb;
      row[2 * d + nt * 16] = vb;
      sk[nt] += bf2f(kb);
      sv[nt] += bf2f(vb);
    }
  }
  if (dbias) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      sk[nt] += __shfl_xor(sk[nt], 16, 64);
      sk[nt] += __shfl_xor(sk[nt], 32, 64);
      sv[nt] += __shfl_xor(sv[nt], 16, 64);
      sv[nt] += __shfl_xor(sv[nt], 32, 64);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      sq[j] += __shfl_xor(sq[j], 16, 64);
      sq[j] += __shfl_xor(sq[j], 32, 64);
    }
    if (lane < 16) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        atomicAdd(dbias + d + h * FD + nt * 16 + lane, sk[nt]);
        atomicAdd(dbias + 2 * d + h * FD + nt * 16 + lane, sv[nt]);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) atomicAdd(dbias + h * FD + (nt0 + j) * 16 + lane, sq[j]);
    }
  }
}

}  // namespace jdt
using namespace jdt;

// S <= 128: the whole-head kernels of attn128.hip (JDT_ATTN128=0 or
// jdt_flash_set_attn128(0): these tile-streaming kernels at every S, for A/B runs)
JDT_API int jdt_attn128_fwd(const void* qkv, void* out, float* lse, int B, int S, int H, float scale, int causal,
                            void* stream);
JDT_API int jdt_attn128_bwd(const void* qkv, const void* out, const void* dout, const float* lse, void* dqkv,
                            float* dbias, int B, int S, int H, float scale, int causal, void* stream);
static int g_attn128 = -1;
static bool attn128_on(int S) {
  if (g_attn128 < 0) {
    const char* e = getenv("JDT_ATTN128");
    g_attn128 = (e && e[0] == '0') ? 0 : 1;
  }
  return g_attn128 && S <= 128;
}
JDT_API void jdt_flash_set_attn128(int on) { g_attn128 = on; }

JDT_API int jdt_flash_fwd(const void* qkv, void* out, float* lse, int B, int S, int H, float scale, int causal,
                          void* stream) {
  if (attn128_on(S)) return jdt_attn128_fwd(qkv, out, lse, B, S, H, scale, causal, stream);
  dim3 grid((S + FB - 1) / FB, B * H);
  hipLaunchKernelGGL(flash_fwd_kernel, grid, dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const bf16_t*>(qkv), static_cast<bf16_t*>(out), lse, S, H, scale, causal);
  return HIP_LAUNCH_CHECK();
}

static bool g_flash_head = true;
JDT_API void jdt_flash_set_head(int on) { g_flash_head = on; }  // A/B: 0 = key-block kernel at every S

// dq_acc: fp32 [B*S, H*64] workspace, all zero on entry and left zero on exit;
// tickets: B*H counters, zero on entry and on exit.
// dbias (optional, fp32 [3*H*64]): += column sums of dQKV (the QKV bias gradient).
JDT_API int jdt_flash_bwd(const void* qkv, const void* out, const void* dout, const float* lse, float* dq_acc,
                          unsigned* tickets, void* dqkv, float* dbias, int B, int S, int H, float scale, int causal,
                          void* stream) {
  if (attn128_on(S)) return jdt_attn128_bwd(qkv, out, dout, lse, dqkv, dbias, B, S, H, scale, causal, stream);
  if (S <= FS && g_flash_head) {  // whole head in one workgroup: dq_acc / tickets untouched (stay zero)
    hipLaunchKernelGGL(flash_bwd_head_kernel, dim3(B * H), dim3(512), 0, static_cast<hipStream_t>(stream),
                       static_cast<const bf16_t*>(qkv), static_cast<const bf16_t*>(out),
                       static_cast<const bf16_t*>(dout), lse, static_cast<bf16_t*>(dqkv), dbias, S, H, scale, causal);
    return HIP_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(flash_bwd_kernel, dim3((S + FB - 1) / FB, B * H), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const bf16_t*>(qkv), static_cast<const bf16_t*>(out),
                     static_cast<const bf16_t*>(dout), lse, static_cast<bf16_t*>(dqkv), dq_acc, tickets, dbias, S, H, scale,
                     causal);
  return HIP_LAUNCH_CHECK();
}
