// Whole-step fused kernels for DEEP tutorial MLPs: 784 -> H -> ... -> H -> C
// (BASELINE configs #2/#3: the 4-layer MLP data-parallel and param-sharded).
//
// The 2-layer classifier runs as 2 launches (mlp_fused.hip).  With L dense
// layers every hidden layer adds one true grid-wide dependency in each
// direction (a row of layer i+1 needs the whole row of layer i), so a step is
// one forward and one backward launch per hidden layer:
//
//   md_fwd (layer i)  grid (row blocks of 16) x (output blocks of 16), 8 waves
//     Z_i = IN W_i + b_i, H_i = dropout(silu(Z_i)); IN is the fp32 data (layer
//     0) or H_{i-1} (bf16).  Also writes IN^T (K-contiguous, for the dW MFMA of
//     the matching backward launch) and the backward factor
//     G_i = silu'(Z_i) * mask/keep, so the backward needs neither Z_i nor Philox.  The last hidden layer also accumulates
//     the head's partial logits H_i[:,blk] W_head[blk,:] with fp32 atomics.
//
//   md_bwd (layer i)  grid (output blocks of 16) x (input chunks of KC), 8 waves
//     dZ_i[:, blk]: TOP (last hidden) from softmax-CE of the summed logits
//     through the head; otherwise (dZ_{i+1} W_{i+1}^T)[:, blk] on MFMA with
//     both fragments loaded straight from global memory -- recomputed by each
//     of the K_IN/KC workgroups of the column block, which is cheaper than a
//     separate launch -- then * G_i (from md_fwd).
//     dW_i[chunk, blk] = IN[:, chunk]^T dZ_i[:, blk] on MFMA (IN^T from md_fwd),
//     db_i (and, TOP, the head's dW/db + metrics) on the spare wave of the
//     chunk-0 workgroups, which also store dZ_i for the next launch.
//     mode 1 (one GPU): AdamW in the epilogue.  W_i's row-major bf16 shadow is
//     still read (old values) by the launch for layer i-1, so it is double
//     buffered by step parity; the K-contiguous copy W_i^T the next forward
//     reads is written directly.  The last launch (layer 0) advances the
//     device step.  mode 0 (N > 1 / FSDP): plain-store grads into the bucket.
//
// Dropout streams match the generic path (models/mlp.py): layer i uses offset
// (i << 1) and 4-row groups (dropout_group), so fused == generic bit-for-bit
// up to summation order.
#include "common.h"

namespace jdt {

constexpr int MD_NT = 512;
constexpr int MD_NW = MD_NT / 64;
constexpr int MD_MPM = 128;  // max rows per device

struct MdArgs {
  int M, K, N, C;       // rows; this layer's in/out features; head classes
  float inv_mb;         // CE grad scale (1 / rows per minibatch)
  const void* X;        // layer input [M][K]: fp32 (layer 0) or bf16
  const bf16_t* Ws0;    // W_i row-major shadow [K][N], step parity 0 / 1 (same pointer if not double buffered)
  const bf16_t* Ws1;
  const bf16_t* WT;     // W_i^T [N][ldwt] (direct fwd fragments) or null -> LDS transposition of Ws
  int ldwt;
  const bf16_t* bs;     // b_i shadow [N]
  float* G;             // backward factor silu'(Z_i) * mask/keep, fp32 [ceil(M/4)][N][4] (dropout-group layout)
  bf16_t* Hout;         // [M][N] activation (next layer's input)
  bf16_t* INT;          // IN^T [K][ldint] (fwd writes, bwd reads)
  int ldint;
  // head (fwd HEAD / bwd TOP)
  const bf16_t* Wh0;    // [N][C] by parity
  const bf16_t* Wh1;
  const bf16_t* bh;     // [C]
  float* logits;        // [2][M][C]
  const int* labels;
  // dropout
  float keep;
  unsigned long long seed, offset;
  int* step;
  unsigned* ticket;
  int advance_step;
  // bwd, !TOP: the next layer
  const bf16_t* dZn;    // dZ_{i+1} [M][NN]
  const bf16_t* Wn0;    // W_{i+1} row-major [N][NN] by parity
  const bf16_t* Wn1;
  bf16_t* dZout;        // dZ_i [M][N] for the launch of layer i-1 (null for layer 0)
  // gradients (mode 0)
  int fuse_opt;
  float* gW; float* gb; float* gWh; float* gbh; float* mslot;
  // AdamW (mode 1)
  float* pW; float* mW; float* vW;
  float* pb; float* mb; float* vb;
  bf16_t* sb;           // b_i shadow out
  bf16_t* WTout;        // W_i^T copy out [N][ldwt]
  float* pWh; float* mWh; float* vWh;
  float* pbh; float* mbh; float* vbh;
  bf16_t* sbh;
  float lr, beta1, beta2, eps, wd, gscale;
  float* running;
  unsigned long long* stamps;   // diagnostic: per-workgroup s_memrealtime at phase ends [grid][8] (null = off)
  // pipeline-stage use (parallel/fused_stage.py)
  int accumulate;       // mode 0: gW/gb/gWh/gbh/mslot += this launch's values (microbatch accumulation)
  const bf16_t* dH;     // bwd BND: gradient w.r.t. this layer's output H_i [M][N] (from the next stage)
  // fwd: the M rows are consecutive microbatches of mb_rows rows (0 = one batch); row
  // r draws its dropout bits from microbatch i = r / mb_rows's own stream -- offset
  // + i * mb_stride, 4-row groups over the microbatch's rows -- exactly the masks a
  // per-microbatch launch (the GPipe microbatch loop) would draw
  int mb_rows;
  unsigned long long mb_stride;
  // mode 0, N > 1: grads + metric slots go to + (step & 1) * stage_stride floats (the
  // xGMI staging half of this step; mlp_fused.hip Mlp2Args::stage_stride)
  long stage_stride;
  // deterministic mode: md_fwd HEAD stores per-column-block partial logits to
  // det_logits[N/16][M][C]; md_bwd TOP sums them in block order (no fp32 atomics)
  float* det_logits;
  // dropout counter high word = step * step_mul (0 or 1: the step): the DP minibatch
  // loop's streams are (step * n_minibatches + i) << 32, i in the offset (dp.py)
  int step_mul;
  // run-ahead (md_bwd AHEAD, layer 0, one GPU, fused AdamW): the layer-0 backward of
  // step t also runs layer 0's forward of step t+1 (mlp_fused.hip Mlp2Args has the
  // same fields): XR row-major bf16 copy of the fp32 input (md_fwd writes it), zslab
  // Z partials [N/16][K/KC][MD_MPM/4][16][4], ztick counters (128-byte lines: step
  // ticket unused here, error word, launch counter; column barriers; per-XCD tile
  // counters), hand = updated b fp32 [N]; G / Hout are layer 0's G_0 / H_0
  bf16_t* XR; float* zslab; unsigned* ztick; float* hand;
  // dZ split (md_bwd, !TOP && !BND, one GPU, every workgroup resident): the K/KC
  // workgroups of a column block each compute only the 16-row blocks w of
  // dZ_i[:, blk] with w % (K/KC) == chunk -- 1/(K/KC) of dZ_{i+1}'s bytes per
  // workgroup instead of all of them -- publish them (write-through) to dzx
  // [N/16][16][MD_MPM] (transposed, as the dzT image) and meet at a per-block arrival
  // counter in dzc (128-byte lines: [0] error word, block b at 32 (1 + b)); then every
  // workgroup reads the whole dZ_i[:, blk] back.  dzs = 0: each workgroup computes all rows.
  bf16_t* dzx; unsigned* dzc; int dzs;
  // mode 0, FSDP N > 1 (accumulate = 0): this layer's gradients + (TOP) head gradients and
  // metric slots straight into the fused FSDP collective's staging buffer (common.h
  // StageMap; leaves W_i, b_i, W_head, b_head, metrics), half = step parity
  const StageMap* smap;
  // bit 0: the dW epilogue's AdamW state (p, m, v) and the K-contiguous bf16 copy are
  // stored write-through (agent-scope sc1) instead of left dirty in the L2 for the
  // kernel boundary to write back (mlp_fused.hip Mlp2Args::wt); bit 1: the row-major
  // bf16 shadow of the next step too
  int wt;
  // N > 1 one-launch-per-layer step: this backward's tiles all-reduce their gradients with
  // the same tiles of the other ranks' launches before the fused AdamW (common.h
  // TxArgs; tile T of this launch is exchange tile tx_base + T; null = one GPU)
  const TxArgs* tx;
  int tx_base;
  int tx_shared;   // ranks share this GPU: the two-workgroups-per-CU variants (jdt_md_tx_ok)
  int tx_fsdp;     // the FSDP form (md_bwd FX): a.pW ... are this rank's LOCAL shards; 2: this
                   // layer's W is sharded along dim 1 (columns; the reference rule for the
                   // square hidden kernels), else along dim 0 (rows)
};

// Slots 0-4: s_memrealtime at the kernel's phase ends (tools/stamp_deep.py).
#define MD_STAMP(i)                                                                          \
  do {                                                                                       \
    if (a.stamps && threadIdx.x == 0)                                                        \
      a.stamps[(long)(blockIdx.y * gridDim.x + blockIdx.x) * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

struct MdAdam { float b1, b2, eps, wd, lr, gs, rbc1, rbc2; };
#ifndef JDT_MD_PIN_ADAM
#define JDT_MD_PIN_ADAM 1
#endif
typedef __attribute__((address_space(1))) unsigned gu32_md;

__device__ __forceinline__ MdAdam md_adam_consts(const MdArgs& a, int step) {
  MdAdam k;
  k.b1 = a.beta1; k.b2 = a.beta2; k.eps = a.eps; k.wd = a.wd; k.lr = a.lr; k.gs = a.gscale;
  const float t = (float)(step + 1);
  k.rbc1 = 1.f / (1.f - powf(a.beta1, t));
  k.rbc2 = 1.f / (1.f - powf(a.beta2, t));
  return k;
}

// write-through (agent-scope sc1) fp32 store: the line is not left dirty in this XCD's L2
__device__ __forceinline__ void md_st(float* p, float v) {
  __hip_atomic_store((__attribute__((address_space(1))) float*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ float md_adam(float p, float m, float v, float g, const MdAdam& k, float* pp, float* mp,
                                         float* vp) {
  g *= k.gs;
  m = k.b1 * m + (1.f - k.b1) * g;
  v = k.b2 * v + (1.f - k.b2) * g * g;
  // v_rcp_f32 (1 ulp) instead of the IEEE divide's scale / fma / fixup sequence, as the
  // 2-layer engine's AdamW (mlp_fused.hip adam_apply)
  p = p - k.lr * ((m * k.rbc1) * __builtin_amdgcn_rcpf(sqrtf(v * k.rbc2) + k.eps) + k.wd * p);
  *pp = p; *mp = m; *vp = v;
  return p;
}

// ---------------------------------------------------------------------------- forward
// DIRECT (compile-time, as in mlp2_fwd): B fragments straight from the W_i^T copy
// (mode 1) instead of an LDS transposition of the row-major shadow (mode 0); a
// runtime branch made the waitcnt pass drain one path's loads at the join.
constexpr int md_fwd_maxt(int k_in) { return ((k_in + 31) / 32 + MD_NW - 1) / MD_NW; }

// A forward tile's operands that do not depend on the layer input (DIRECT: the W_i^T
// fragments of this wave's k range, the bias, the head weight): loaded before the input is
// ready when the tile is the second of a fused pair (md_fwd2_kernel).
template <int MAXT> struct MdFwdPre { bf16x8 bg[MAXT]; float whv, bv; };

template <int K_IN, bool HEAD, int C>
__device__ __forceinline__ void md_fwd_wload(const MdArgs& a, int by, int step, MdFwdPre<md_fwd_maxt(K_IN)>& P) {
  constexpr int NW = MD_NW, KS = (K_IN + 31) / 32, MAXT = md_fwd_maxt(K_IN);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int j0 = by * 16, par = step & 1;
  const int ks0 = (w * KS) / NW, ks1 = ((w + 1) * KS) / NW;
  // every load unconditional (clamped address; out-of-range values are never used or
  // are zeroed at the LDS write): a load under a divergent guard is waited for at the join
#pragma unroll
  for (int t = 0; t < MAXT; ++t) {
    const int ks = min(ks0 + t, ks1 - 1);
    P.bg[t] = *reinterpret_cast<const bf16x8*>(a.WT + (long)(j0 + (lane & 15)) * a.ldwt + ks * 32 + 8 * (lane >> 4));
  }
  const bf16_t* Wh = par ? a.Wh1 : a.Wh0;
  P.whv = HEAD ? bf2f(Wh[(long)(j0 + min(tid, 16 * C - 1) / C) * C + min(tid, 16 * C - 1) % C]) : 0.f;
  P.bv = bf2f(a.bs[j0 + (tid & 15)]);
}

// FM (md_fwd2_kernel, two consecutive hidden layers in one launch): 0 = a standalone
// launch; 1 = the pair's first layer -- its H rows also leave write-through (sc1) for the
// second layer's workgroups; 2 = the pair's second layer -- its input X (the first layer's
// H) loaded sc1, the input-independent operands taken from `pre`.
template <int K_IN, bool XF32, int XTC, bool HEAD, int C, int RB, bool DIRECT, int FM = 0>
__device__ __forceinline__ void md_fwd_body(const MdArgs& a, const int bx, const int by,
                                            const MdFwdPre<md_fwd_maxt(K_IN)>* pre) {
  constexpr int NT = MD_NT, NW = MD_NW;
  constexpr int KS = (K_IN + 31) / 32;
  constexpr int KP = KS * 32;
  constexpr int LDW = KP + 8;
  constexpr int WCH = (K_IN * 2 + NT - 1) / NT;   // 16-byte W chunks per thread (LDS path)
  constexpr int MAXT = md_fwd_maxt(K_IN);
  constexpr int LDXS = K_IN + 8;
  static_assert(K_IN % XTC == 0 && XTC % 8 == 0 && XTC * 4 <= NT && K_IN % 8 == 0, "IN^T chunking");
  static_assert(FM == 0 || (DIRECT && !XF32 && RB == 16), "fused pair: bf16 input, W^T fragments, 16-row blocks");
  __shared__ __attribute__((aligned(16))) bf16_t wt[DIRECT ? 8 : 16 * LDW];
  __shared__ __attribute__((aligned(16))) bf16_t xs[RB * LDXS];
  __shared__ float part[NW][RB][17];
  __shared__ float htile[RB][17];
  __shared__ float whs[16][C > 0 ? C : 1];
  __shared__ float bsh[16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int M = a.M, N = a.N;
  const int r0 = bx * RB, j0 = by * 16;
  const int step = a.step[0], par = step & 1;
  const unsigned long long doff =
      a.offset + ((unsigned long long)(unsigned)(a.step_mul > 1 ? step * a.step_mul : step) << 32);
  const bf16_t* Ws = par ? a.Ws1 : a.Ws0;
  const int ks0 = (w * KS) / NW, ks1 = ((w + 1) * KS) / NW;
  constexpr bool direct = DIRECT;

  // ---- 1. every global load up front
  u32x4 wv[WCH];
  MdFwdPre<MAXT> P;
  if constexpr (!DIRECT) {
#pragma unroll
    for (int t = 0; t < WCH; ++t) {
      const int idx = min(tid + t * NT, K_IN * 2 - 1);
      wv[t] = *reinterpret_cast<const u32x4*>(Ws + (long)(idx >> 1) * N + j0 + (idx & 1) * 8);
    }
  } else if constexpr (FM != 2) {
    md_fwd_wload<K_IN, HEAD, C>(a, by, step, P);
  }
  if constexpr (FM == 2) P = *pre;
  // input row block [RB][K_IN], coalesced 16-byte loads (FM 2: sc1, the hand-off of the
  // pair's first layer, past this CU's L1 and any stale L2 line)
  constexpr int EPV = XF32 ? 4 : 8;                 // elements per 16-byte vector
  constexpr int XV = RB * K_IN / EPV;
  constexpr int XPT = (XV + NT - 1) / NT;
  u32x4 xv[XPT];
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.X), (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
  for (int e = 0; e < XPT; ++e) {
    const int f = min(tid + e * NT, XV - 1), rl = f / (K_IN / EPV), kv = f % (K_IN / EPV);
    const long off = ((long)min(r0 + rl, M - 1) * K_IN + (long)kv * EPV) * (XF32 ? 4 : 2);
    if constexpr (FM == 2)
      xv[e] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, (int)off, 0, 16));
    else
      xv[e] = *reinterpret_cast<const u32x4*>(static_cast<const char*>(a.X) + off);
  }
  const bf16x8* bg = P.bg;
  const float whv = DIRECT ? P.whv
                           : (HEAD ? bf2f((par ? a.Wh1 : a.Wh0)[(long)(j0 + min(tid, 16 * C - 1) / C) * C +
                                                              min(tid, 16 * C - 1) % C])
                                   : 0.f);
  const float bv = DIRECT ? P.bv : bf2f(a.bs[j0 + (tid & 15)]);

  // ---- 2. LDS images
  if (!direct) {
#pragma unroll
    for (int t = 0; t < WCH; ++t) {
      const int idx = tid + t * NT;
      if (idx < K_IN * 2) {
        const int k = idx >> 1, h = (idx & 1) * 8;
        const unsigned q[4] = {wv[t].x, wv[t].y, wv[t].z, wv[t].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          wt[(h + 2 * e) * LDW + k] = (bf16_t)(q[e] & 0xffff);
          wt[(h + 2 * e + 1) * LDW + k] = (bf16_t)(q[e] >> 16);
        }
      }
    }
    if (KP > K_IN)
      for (int idx = tid; idx < 16 * (KP - K_IN); idx += NT) wt[(idx / (KP - K_IN)) * LDW + K_IN + idx % (KP - K_IN)] = 0;
  }
  if (HEAD && tid < 16 * C) whs[tid / C][tid % C] = whv;
  if (tid < 16) bsh[tid] = bv;
#pragma unroll
  for (int e = 0; e < XPT; ++e) {
    const int f = tid + e * NT, rl = f / (K_IN / EPV), kv = f % (K_IN / EPV);
    if (f < XV) {
      const bool ok = r0 + rl < M;   // rows past M stay zero (IN^T tail is read by md_bwd)
      if (XF32) {
        const float4 x = *reinterpret_cast<const float4*>(&xv[e]);
        *reinterpret_cast<uint2*>(&xs[rl * LDXS + 4 * kv]) =
            ok ? make_uint2((unsigned)f2bf(x.x) | ((unsigned)f2bf(x.y) << 16),
                            (unsigned)f2bf(x.z) | ((unsigned)f2bf(x.w) << 16))
               : make_uint2(0u, 0u);
      } else {
        *reinterpret_cast<u32x4*>(&xs[rl * LDXS + 8 * kv]) = ok ? xv[e] : (u32x4){0u, 0u, 0u, 0u};
      }
    }
  }
  __syncthreads();
  // IN^T side output: output block y < K_IN/XTC writes features [y*XTC, (y+1)*XTC) of this row block
  if (a.INT && by < K_IN / XTC && tid < XTC * (RB / 8)) {
    const int i = tid / (RB / 8), h = (tid % (RB / 8)) * 8, xk = by * XTC + i;
    unsigned q[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      q[e] = (unsigned)xs[(h + 2 * e) * LDXS + xk] | ((unsigned)xs[(h + 2 * e + 1) * LDXS + xk] << 16);
    u32x4 o; o.x = q[0]; o.y = q[1]; o.z = q[2]; o.w = q[3];
    *reinterpret_cast<u32x4*>(a.INT + (long)xk * a.ldint + r0 + h) = o;
  }
  // row-major bf16 input (run-ahead layer-0 backward: the next step's forward operand)
  if (XF32 && a.XR && by < K_IN / XTC && tid < RB * (XTC / 8)) {
    const int rl = tid / (XTC / 8), q = tid % (XTC / 8);
    if (r0 + rl < M)
      *reinterpret_cast<u32x4*>(a.XR + (long)(r0 + rl) * K_IN + by * XTC + 8 * q) =
          *reinterpret_cast<const u32x4*>(&xs[rl * LDXS + by * XTC + 8 * q]);
  }

  // ---- 3. K split over the 8 waves
  constexpr int MT = RB / 16;
  f32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < MAXT; ++t) {
    if (ks0 + t < ks1) {
      const int k = (ks0 + t) * 32 + 8 * (lane >> 4);
      const bf16x8 b = direct ? bg[t] : *reinterpret_cast<const bf16x8*>(&wt[(lane & 15) * LDW + k]);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        bf16x8 af = (bf16x8){0, 0, 0, 0, 0, 0, 0, 0};
        if (k < K_IN) af = *reinterpret_cast<const bf16x8*>(&xs[(mt * 16 + (lane & 15)) * LDXS + k]);
        acc[mt] = mfma16x16x32(af, b, acc[mt]);
      }
    }
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int e = 0; e < 4; ++e) part[w][mt * 16 + (lane >> 4) * 4 + e][lane & 15] = acc[mt][e];
  __syncthreads();

  // ---- 4. bias + silu + dropout per 4-row group
  if (tid < (RB / 4) * 16) {
    const int g4 = tid >> 4, c = tid & 15, col = j0 + c;
    const int rowg = r0 + g4 * 4;
    u32x4 db = {0u, 0u, 0u, 0u};
    if (a.keep < 1.f && rowg < M) {
      int lrow = rowg, Mg = M;
      unsigned long long off = doff;
      if (a.mb_rows > 0) {   // mb_rows % 4 == 0: a 4-row group never straddles microbatches
        const int mi = rowg / a.mb_rows;
        lrow = rowg - mi * a.mb_rows;
        Mg = a.mb_rows;
        off += (unsigned long long)mi * a.mb_stride;
      }
      db = dropout_bits(a.seed, off, dropout_group(0, lrow, col, Mg, N));
    }
    float gf[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int rl = g4 * 4 + e, row = r0 + rl;
      float hv = 0.f;
      gf[e] = 0.f;
      if (row < M) {
        float v = bsh[c];
#pragma unroll
        for (int q = 0; q < NW; ++q) v += part[q][rl][c];
        const float z = bf2f(f2bf(v));           // Z_i as the bf16 Dense output
        const float ez = __expf(-z);
        const float sg = 1.0f / (1.0f + ez);
        hv = z * sg;                             // act_fwd(ACT_SILU)
        float gd = sg * (1.0f + z * (1.0f - sg));  // act_grad(ACT_SILU)
        if (a.keep < 1.f) {
          const bool kp = keep_word(db, e, a.keep);
          hv = kp ? hv / a.keep : 0.f;
          gd = kp ? gd / a.keep : 0.f;
        }
        gf[e] = gd;
        const bf16_t hb = f2bf(hv);
        if constexpr (FM != 1) a.Hout[(long)row * N + col] = hb;
        hv = bf2f(hb);
      }
      htile[rl][c] = hv;
    }
    *reinterpret_cast<float4*>(a.G + ((long)(rowg >> 2) * N + col) * 4) = make_float4(gf[0], gf[1], gf[2], gf[3]);
  }
  if constexpr (FM == 1) {
    // the H tile as 16-byte write-through rows (the pair's second layer reads them across
    // workgroups within this launch): 16 rows x 2 halves of 8 columns
    __syncthreads();
    if (tid < 2 * RB) {
      const int rl = tid >> 1, h8 = (tid & 1) * 8, row = r0 + rl;
      unsigned q[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        q[e] = (unsigned)f2bf(htile[rl][h8 + 2 * e]) | ((unsigned)f2bf(htile[rl][h8 + 2 * e + 1]) << 16);
      const __amdgpu_buffer_rsrc_t hr =
          __builtin_amdgcn_make_buffer_rsrc(a.Hout, (short)0, M * N * 2, 0x00020000);
      // rows past M: out of the resource's range, dropped
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned,
                                                                (u32x4){q[0], q[1], q[2], q[3]}),
                                             hr, (int)(((long)row * N + j0 + h8) * 2), 0, 16);
    }
  }
  if (HEAD) {
    __syncthreads();
    float* lg = a.logits + (long)par * M * C;
    if (tid < RB * C) {
      const int rl = tid / C, c = tid % C, row = r0 + rl;
      if (row < M) {
        float s = (by == 0) ? bf2f(a.bh[c]) : 0.f;
#pragma unroll
        for (int n = 0; n < 16; ++n) s += htile[rl][n] * whs[n][c];
        if (a.det_logits) a.det_logits[((long)by * M + row) * C + c] = s;
        else atomicAdd(lg + (long)row * C + c, s);
      }
    }
  }
}

template <int K_IN, bool XF32, int XTC, bool HEAD, int C, int RB, bool DIRECT, bool XCD>
__global__ void __launch_bounds__(MD_NT) md_fwd_kernel(MdArgs a) {
  int bx = blockIdx.x, by = blockIdx.y;
  // XCD-contiguous: each XCD takes 4 whole column blocks (1/8 of W_i) over all row blocks
  if constexpr (XCD) xcd_contiguous_tile(bx, by);
  md_fwd_body<K_IN, XF32, XTC, HEAD, C, RB, DIRECT>(a, bx, by, nullptr);
}

// Two consecutive 512 -> 512 hidden layers' forwards in ONE launch (the 4-layer MLP's
// layers 1 and 2 + the head logits; layer 0 runs ahead in the previous step's layer-0
// backward): workgroup (r, c) computes tile (r, c) of layer i, then -- once the 32
// workgroups of its 16-row block have stored their H_i tiles (write-through) and added to
// the block's arrival counter -- tile (r, c) of layer i+1 from those 16 rows (sc1 loads).
// A row of layer i+1 needs only the same row of layer i, so the launch boundary between
// the two layers becomes a 32-workgroup counter per row block; the second layer's W^T
// fragments, bias and head weight are loaded before the wait.  rowc: 128-byte lines,
// [0] error word (bit 0: a row block's wait timed out -- not every workgroup resident),
// block r's monotonic counter at 32 (1 + r).  Requires every workgroup resident
// (jdt_md_fwd2_ok).
__global__ void __launch_bounds__(MD_NT) md_fwd2_kernel(MdArgs a1, MdArgs a2, unsigned* rowc) {
  const int bx = blockIdx.x, by = blockIdx.y;
  MdFwdPre<md_fwd_maxt(512)> pre;
  md_fwd_wload<512, true, 10>(a2, by, a2.step[0], pre);
  md_fwd_body<512, false, 16, false, 10, 16, true, 1>(a1, bx, by, nullptr);
  // every wave's write-through H stores have left, then one arrival per workgroup; a launch
  // adds gridDim.y per block, so the target is the next multiple above this arrival
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned* cnt = rowc + 32 * (1 + bx);
    const unsigned nb = gridDim.y;
    const unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned target = (old / nb + 1u) * nb;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const __amdgpu_buffer_rsrc_t cr = __builtin_amdgcn_make_buffer_rsrc(cnt, (short)0, 4, 0x00020000);
    while ((int)((unsigned)__builtin_amdgcn_raw_buffer_load_b32(cr, 0, 0, 16) - target) < 0) {
      if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > 2000000ll) {   // 20 ms: a block-mate never ran
        atomicOr(rowc, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      asm volatile("" ::: "memory");
    }
  }
  __syncthreads();
  md_fwd_body<512, false, 16, true, 10, 16, true, 2>(a2, bx, by, &pre);
}

// ---------------------------------------------------------------------------- backward
// BND (pipeline stage boundary, !TOP): dZ_i = dH * G_i -- the gradient w.r.t. this
// layer's output arrives from the next pipeline stage instead of being recomputed
// from dZ_{i+1} W_{i+1}^T.
// TX: N > 1, in-kernel tile exchange.  WPE = 4 (two workgroups per CU, <= 128 VGPRs,
// a few spills) is the variant for ranks SHARING one GPU -- both ranks' launches must be
// resident at once for the exchange's waits (jdt_md_tx_ok); with a GPU per rank one
// workgroup per CU suffices and WPE = 1 keeps the unconstrained allocation.
// FX (with TX): the FSDP form -- every gradient element goes to the rank that owns its
// row (the reference's dim-0 shards), the owner applies the SHARDED AdamW on its local
// state and hands the updated value back (as mlp_fused.hip mlp2_bwd FX).
template <int K_IN, bool TOP, int C, int KC, int NN, bool XCD, bool BND = false, bool AHEAD = false, bool TX = false,
          int WPE = 1, bool FX = false>
__global__ void __launch_bounds__(MD_NT) __attribute__((amdgpu_waves_per_eu(WPE))) md_bwd_kernel(MdArgs a) {
  constexpr int NT = MD_NT, NW = MD_NW, MPM = MD_MPM;
  constexpr int LDM = MPM + 8;
  constexpr int NTILE = KC / 16;           // dW output tiles (one per wave)
  constexpr int NKS = NN / 32;             // k-steps of the dZ_{i+1} W_{i+1}^T product
  static_assert(KC % 16 == 0 && K_IN % KC == 0 && NTILE <= NW - 1, "tile plan");
  static_assert(!FX || (TX && !BND), "FX is the FSDP form of the exchanging backward");
  static_assert((MPM / 4) * 16 == NT, "one 4-row group per thread");
  __shared__ float dlog[TOP ? MPM : 1][C + 1];
  __shared__ __attribute__((aligned(16))) bf16_t dzT[16 * LDM];
  __shared__ __attribute__((aligned(16))) bf16_t hT[16 * LDM];     // H_i[:, blk]^T (TOP, chunk-0)
  __shared__ __attribute__((aligned(16))) bf16_t dlT[16 * LDM];    // dlogits^T (TOP)
  __shared__ float whs[16][C];
  __shared__ float red[2][NW];
  // !TOP: W_{i+1}[blk, :] staged once per workgroup (it used to be loaded by every
  // wave: 8 x 16 KB of the per-CU intake, which bounds this phase -- stamps);
  // rows padded by 16 B so the 16 rows of a B fragment read hit distinct banks
  constexpr int LDWN = NN + 8;
  constexpr int WNCH = 16 * NN / 8;                    // 16-byte chunks of the tile
  static_assert(TOP || WNCH % MD_NT == 0, "Wn tile chunking");
  static_assert(!(TOP && BND), "TOP and BND are exclusive");
  constexpr bool WN = !TOP && !BND;   // dZ_i from the next layer of this launch sequence
  __shared__ __attribute__((aligned(16))) bf16_t wnS[WN ? 16 * LDWN : 8];
  // run-ahead (layer 0): W_0'[chunk, blk]^T image for the next forward's partial, H tile
  static_assert(!AHEAD || (WN && K_IN == 784 && KC <= 128 && KC % 16 == 0), "run-ahead: layer 0 only");
  constexpr int LDW1 = 128 + 8;
  constexpr int NCH = K_IN / KC;
  __shared__ __attribute__((aligned(16))) bf16_t w1n[AHEAD ? 16 * LDW1 : 8];
  // the wave index through readfirstlane: the compiler then knows it is wave-uniform, so
  // the per-wave buffer resources below (dZ split) stay scalar -- derived from threadIdx it
  // is a VGPR, and every buffer access through it became a readfirstlane waterfall loop
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int M = a.M, N = a.N, Mp = (M + 31) & ~31;
  int bx = blockIdx.x, by = blockIdx.y;
  if constexpr (AHEAD) xcd_column_tile(bx, by);      // a column block on ONE XCD (common.h)
  else if constexpr (XCD) xcd_contiguous_tile(bx, by);   // column-block neighbours share an L2 (common.h)
  const int j0 = bx * 16, kc0 = by * KC;
  const bool chunk0 = by == 0;
  const bool lead = TOP && bx == 0 && by == 0;
  const int rg = tid >> 4, gn = tid & 15;   // TOP: this thread's group (rows 4rg..4rg+3, column j0+gn)
  const bool dzs = WN && a.dzs != 0;
  const bool act = !dzs || (w % NCH) == by;   // wave-uniform: this wave computes its 16 dZ rows

  MD_STAMP(0);
  // ---- 0. every global load up front, all unconditional (clamped addresses: values
  // of rows past M or outside this wave's role are never used) and both step
  // parities of the parity-buffered operands, so nothing waits on the step counter,
  // which is loaded last, per lane (a uniform load is read back through
  // readfirstlane, which would wait for every load in flight), and selects them.
  const bool fo = a.fuse_opt != 0;
  int lz;
  asm volatile("v_mov_b32 %0, 0" : "=v"(lz));
  // !TOP: the step counter is loaded FIRST (only W_{i+1}'s parity buffer depends on
  // it, and those loads are issued last, after one round trip); TOP: last.
  int step = 0;
  if constexpr (WN) {
    step = a.step[lz];
    __builtin_amdgcn_sched_barrier(0);
  }
  float lr0[TOP ? C : 1], lr1[TOP ? C : 1];
  int lab = 0;
  float4 gv;
  bf16_t hv[4];
  bf16x8 dzf[WN ? NKS : 1];
  u32x4 wq[WN ? WNCH / MD_NT : 1];
  unsigned long long dhq = 0;
  float whv0 = 0.f, whv1 = 0.f;
  if constexpr (TOP) {
    const long lo = (long)min(tid, M - 1) * C;
    if (a.det_logits) {
#pragma unroll
      for (int c = 0; c < C; ++c) lr0[c] = 0.f;
      for (int q = 0; q < N / 16; ++q) {
        const float* pq = a.det_logits + (long)q * M * C + lo;
#pragma unroll
        for (int c = 0; c < C; ++c) lr0[c] += pq[c];
      }
#pragma unroll
      for (int c = 0; c < C; ++c) lr1[c] = lr0[c];
    } else {
#pragma unroll
      for (int c = 0; c < C; ++c) { lr0[c] = a.logits[lo + c]; lr1[c] = a.logits[(long)M * C + lo + c]; }
    }
    lab = a.labels[min(tid, M - 1)];
    gv = *reinterpret_cast<const float4*>(a.G + ((long)min(rg, (M - 1) >> 2) * N + j0 + gn) * 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) hv[e] = a.Hout[(long)min(rg * 4 + e, M - 1) * N + j0 + gn];
    const int wi = min(tid, 16 * C - 1);
    const long wo = (long)(j0 + wi / C) * C + wi % C;
    whv0 = bf2f(a.Wh0[wo]);
    whv1 = bf2f(a.Wh1[wo]);
  } else if constexpr (BND) {
    // wave w, lane: rows 16w + 4(lane>>4) .. +3 of column j0 + (lane&15) of dH and G
    const int row0 = w * 16 + (lane >> 4) * 4, col = j0 + (lane & 15);
#pragma unroll
    for (int e = 0; e < 4; ++e)
      dhq |= (unsigned long long)a.dH[(long)min(row0 + e, M - 1) * N + col] << (16 * e);
    gv = *reinterpret_cast<const float4*>(a.G + ((long)(min(row0, M - 1) >> 2) * N + col) * 4);
  } else {
    // wave w: rows 16w..16w+15 of dZ_i[:, blk] = dZ_{i+1} . W_{i+1}[blk, :]^T
    const int row = min(w * 16 + (lane & 15), M - 1);
    // a wave that skips its rows (dZ split) gets a zero-length resource: its loads
    // return zeros without a memory access and without a branch around them
    const __amdgpu_buffer_rsrc_t dzr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16_t*>(a.dZn), (short)0, act ? M * NN * 2 : 0, 0x00020000);
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
      dzf[ks] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                               dzr, (int)(((long)row * NN + ks * 32 + 8 * (lane >> 4)) * 2), 0, 0));
    const int row0 = min(w * 16 + (lane >> 4) * 4, M - 1);
    gv = *reinterpret_cast<const float4*>(a.G + ((long)(row0 >> 2) * N + j0 + (lane & 15)) * 4);
  }
  // A fragments of this wave's dW tile from IN^T (zero-padded to Mp samples)
  const int wt_ = min(w, NTILE - 1);
  bf16x8 xf[MPM / 32];
#pragma unroll
  for (int ks = 0; ks < MPM / 32; ++ks)
    xf[ks] = *reinterpret_cast<const bf16x8*>(a.INT + (long)(kc0 + wt_ * 16 + (lane & 15)) * a.ldint +
                                              min(ks, Mp / 32 - 1) * 32 + 8 * (lane >> 4));
  // AdamW state of this lane's outputs (mode 0 has none: the loads then read the
  // gradient buffers, values unused).  Waves < NTILE: their dW tile; the aux wave
  // (chunk-0 blocks): the head's dW rows (TOP) in op/om/ov and b_i in bp/bm/bvv.
  float op[4], om[4], ov[4];
  const int trow0 = kc0 + wt_ * 16 + (lane >> 4) * 4;
  const int tcol = j0 + (lane & 15);
  const bool aux = chunk0 && w == NW - 1;
  const int ac = lane & 15;
  float bp[4], bm[4], bvv[4], qp = 0.f, qm = 0.f, qv = 0.f;
  // FX: this rank R of W owns W rows [R K/W, (R+1) K/W) and bias / head rows
  // [R N/W, (R+1) N/W); its AdamW state (a.pW ... a.vbh) is that LOCAL shard
  int fx_R = 0, fx_W = 1, fx_rpq = K_IN, fx_hpq = 512;
  bool fx_col = false;   // W column-sharded: the whole tile has one owner (j0 / hpq)
  if constexpr (FX) {
    fx_R = __builtin_amdgcn_readfirstlane(a.tx->rank);
    fx_W = __builtin_amdgcn_readfirstlane(a.tx->world);
    fx_rpq = K_IN / fx_W;
    fx_hpq = N / fx_W;
    fx_col = __builtin_amdgcn_readfirstlane(a.tx_fsdp) == 2;
  }
  {
    const bool hw = TOP && aux;   // wave-uniform
    const float* sp = hw ? (fo ? a.pWh : a.gWh) : (fo ? a.pW : a.gW);
    const float* sm = hw ? (fo ? a.mWh : a.gWh) : (fo ? a.mW : a.gW);
    const float* sv = hw ? (fo ? a.vWh : a.gWh) : (fo ? a.vW : a.gW);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int n = (lane >> 4) * 4 + e;
      // (FX: clamped into the local shard; values of rows this rank does not own unused)
      const int hrow = FX ? min(max(j0 + n - fx_R * fx_hpq, 0), fx_hpq - 1) : j0 + n;
      const int wrow = (FX && !fx_col) ? min(max(trow0 + e - fx_R * fx_rpq, 0), fx_rpq - 1) : trow0 + e;
      const long idx = hw ? (long)hrow * C + min(ac, C - 1)
                          : (FX && fx_col) ? (long)wrow * fx_hpq + min(max(tcol - fx_R * fx_hpq, 0), fx_hpq - 1)
                                           : (long)wrow * N + tcol;
      op[e] = sp[idx]; om[e] = sm[idx]; ov[e] = sv[idx];
      const float* bq = fo ? a.pb : a.gb;
      const float* bmq = fo ? a.mb : a.gb;
      const float* bvq = fo ? a.vb : a.gb;
      bp[e] = bq[hrow]; bm[e] = bmq[hrow]; bvv[e] = bvq[hrow];
    }
    if constexpr (TOP) {
      const int lq = min(lane, C - 1);
      qp = (fo ? a.pbh : a.gbh)[lq]; qm = (fo ? a.mbh : a.gbh)[lq]; qv = (fo ? a.vbh : a.gbh)[lq];
    }
  }
  // run-ahead: X[16w.., chunk] fragments for the next forward (in flight through the
  // backward); this thread's epilogue element: row group eg of the share [g_lo, g_hi)
  // of this chunk, column j0 + gn (its dropout bits dbn are computed in phase 5)
  bf16x8 xa[AHEAD ? 4 : 1];
  u32x4 dbn = {0u, 0u, 0u, 0u};
  const int g_lo = (by * (MPM / 4)) / NCH, g_hi = ((by + 1) * (MPM / 4)) / NCH;
  const int eg = g_lo + (tid >> 6), ee = (tid >> 4) & 3;
  if constexpr (AHEAD) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
      xa[ks] = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(
                   a.XR + (long)min(w * 16 + (lane & 15), M - 1) * K_IN + min(kc0 + ks * 32 + 8 * (lane >> 4), K_IN - 8)));
    for (int idx = tid; idx < 16 * (128 - KC); idx += NT) w1n[(idx / (128 - KC)) * LDW1 + KC + idx % (128 - KC)] = 0;
  }
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (!WN) step = a.step[lz];
  const int par = step & 1;
  if constexpr (WN) {
    const bf16_t* Wn = par ? a.Wn1 : a.Wn0;
#pragma unroll
    for (int t = 0; t < WNCH / MD_NT; ++t) {
      const int c = tid + t * MD_NT;
      wq[t] = *reinterpret_cast<const u32x4*>(Wn + (long)(j0 + c / (NN / 8)) * NN + (c % (NN / 8)) * 8);
    }
  }
  float lrow[TOP ? C : 1];
  float whv = 0.f;
  if constexpr (TOP) {
#pragma unroll
    for (int c = 0; c < C; ++c) lrow[c] = par ? lr1[c] : lr0[c];
    whv = par ? whv1 : whv0;
  }
  const MdAdam ak = md_adam_consts(a, step);
  // the bias corrections (two powf + two divides per lane) here, before the phase-1 work:
  // left to the compiler they sink to the AdamW epilogue, on the critical path behind the
  // MFMAs (the persistent headline kernel's lesson, profiles/r5_pst_headline.txt)
  // (JDT_MD_PIN_ADAM: 1 every layer, 2 only where the step counter is the first load (!TOP)).
  // Not in the N > 1 exchange variants: two more live registers put the top layer's TX
  // variant at 133 VGPRs, one workgroup per CU, and 2 ranks' grids no longer co-resident
  if (!TX && (JDT_MD_PIN_ADAM == 1 || (JDT_MD_PIN_ADAM == 2 && WN))) asm volatile("" ::"v"(ak.rbc1), "v"(ak.rbc2));
  const long goff = (!fo && a.stage_stride) ? (long)par * a.stage_stride : 0;   // staged bucket half

  MD_STAMP(1);
  // ---- 1/2. dZ_i[:, blk] -> dzT[n][m] (bf16), dZout (chunk-0)
  float l_loss = 0.f, l_corr = 0.f;
  if constexpr (TOP) {
    if (tid < M) {
      float mx = -INFINITY;
      int am = 0;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        lrow[c] = round_bf(lrow[c]);
        if (lrow[c] > mx) { mx = lrow[c]; am = c; }
      }
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < C; ++c) s += __expf(lrow[c] - mx);
      const float lse = mx + __logf(s);
      l_loss = lse - lrow[lab];
      l_corr = (am == lab) ? 1.f : 0.f;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const bf16_t gb = f2bf((__expf(lrow[c] - lse) - (c == lab ? 1.f : 0.f)) * a.inv_mb);
        dlog[tid][c] = bf2f(gb);
        dlT[c * LDM + tid] = gb;
      }
    } else if (tid < MPM) {
#pragma unroll
      for (int c = 0; c < C; ++c) dlT[c * LDM + tid] = 0;
    }
    for (int idx = tid; idx < (16 - C) * MPM; idx += NT) dlT[(C + idx / MPM) * LDM + idx % MPM] = 0;
    if (tid < 16 * C) whs[tid / C][tid % C] = whv;   // whv: this step's parity
    if (lead) {
      l_loss = wave_sum(l_loss);
      l_corr = wave_sum(l_corr);
      if (lane == 0) { red[0][w] = l_loss; red[1][w] = l_corr; }
      float* nxt = a.logits + (long)(par ^ 1) * M * C;   // re-arm next step's accumulator
      for (int i = tid; i < M * C; i += NT) nxt[i] = 0.f;
    }
    __syncthreads();
    const float gfac[4] = {gv.x, gv.y, gv.z, gv.w};
    unsigned packed[2] = {0u, 0u};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int m = rg * 4 + e;
      float v = 0.f;
      if (m < M) {
        float dh = 0.f;
#pragma unroll
        for (int c = 0; c < C; ++c) dh += dlog[m][c] * whs[gn][c];
        v = dh * gfac[e];
      }
      const bf16_t vb = f2bf(v);
      packed[e >> 1] |= (unsigned)vb << (16 * (e & 1));
      if (chunk0 && a.dZout && m < M) a.dZout[(long)m * N + j0 + gn] = vb;
    }
    *reinterpret_cast<uint2*>(&dzT[gn * LDM + rg * 4]) = make_uint2(packed[0], packed[1]);
    if (chunk0)
      *reinterpret_cast<uint2*>(&hT[gn * LDM + rg * 4]) =
          make_uint2((unsigned)hv[0] | ((unsigned)hv[1] << 16), (unsigned)hv[2] | ((unsigned)hv[3] << 16));
  } else {
    if constexpr (WN) {
#pragma unroll
      for (int t = 0; t < WNCH / MD_NT; ++t) {
        const int c = tid + t * MD_NT;
        *reinterpret_cast<u32x4*>(&wnS[(c / (NN / 8)) * LDWN + (c % (NN / 8)) * 8]) = wq[t];
      }
      __syncthreads();
    }
    if (w * 16 < Mp && act) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      if constexpr (WN) {
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          const bf16x8 wnf = *reinterpret_cast<const bf16x8*>(&wnS[(lane & 15) * LDWN + ks * 32 + 8 * (lane >> 4)]);
          acc = mfma16x16x32(dzf[ks], wnf, acc);
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] = bf2f((bf16_t)(dhq >> (16 * e)));
      }
      const int row0 = w * 16 + (lane >> 4) * 4, col = j0 + (lane & 15);
      const float gfac[4] = {gv.x, gv.y, gv.z, gv.w};
      unsigned packed[2] = {0u, 0u};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = row0 + e;
        float v = 0.f;
        if (m < M) {
          v = acc[e] * gfac[e];
        }
        const bf16_t vb = f2bf(v);
        packed[e >> 1] |= (unsigned)vb << (16 * (e & 1));
        if ((dzs || chunk0) && a.dZout && m < M) a.dZout[(long)m * N + col] = vb;
      }
      *reinterpret_cast<uint2*>(&dzT[(lane & 15) * LDM + row0]) = make_uint2(packed[0], packed[1]);
      if (dzs) {   // publish (write-through) for the block's other workgroups
        const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(a.dzx + (long)bx * 16 * MPM, (short)0,
                                                                            16 * MPM * 2, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned,
                                                                 make_uint2(packed[0], packed[1])),
                                              xr, ((lane & 15) * MPM + row0) * 2, 0, 16);
      }
    }
  }
  __syncthreads();
  if (dzs) {
    // every wave's exchange stores have left (sc1: at the coherence point), then one
    // arrival per workgroup; a launch adds NCH per block, so the target is the next
    // multiple of NCH above this workgroup's own arrival ticket
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      unsigned* cnt = a.dzc + 32 * (1 + bx);
      const unsigned old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (old / NCH + 1u) * NCH;
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      const __amdgpu_buffer_rsrc_t cr = __builtin_amdgcn_make_buffer_rsrc(cnt, (short)0, 4, 0x00020000);
      while ((int)((unsigned)__builtin_amdgcn_raw_buffer_load_b32(cr, 0, 0, 16) - target) < 0) {
        if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > 2000000ll) {   // 20 ms: a block-mate never ran
          atomicOr(a.dzc, 1u);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");
      }
    }
    __syncthreads();
    // the whole dZ_i[:, blk]^T back into dzT (16-byte sc1 loads, past this CU's L1)
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(a.dzx + (long)bx * 16 * MPM, (short)0,
                                                                        16 * MPM * 2, 0x00020000);
    for (int c = tid; c < 16 * (Mp / 8); c += NT) {
      const int n = c / (Mp / 8), r8 = (c % (Mp / 8)) * 8;
      const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(xr, (n * MPM + r8) * 2, 0, 16));
      *reinterpret_cast<u32x4*>(&dzT[n * LDM + r8]) = v;
    }
    __syncthreads();
  }

  MD_STAMP(2);
  // ---- 3. dW_i[chunk, blk] = IN[:, chunk]^T dZ_i[:, blk]; spare wave: db_i (+ head grads)
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  f32x4 aw = {0.f, 0.f, 0.f, 0.f}, ab = {0.f, 0.f, 0.f, 0.f}, ab2 = {0.f, 0.f, 0.f, 0.f};
  if (w < NTILE) {
#pragma unroll
    for (int ks = 0; ks < MPM / 32; ++ks) {
      if (ks < Mp / 32) {
        const int kk = ks * 32 + 8 * (lane >> 4);
        const bf16x8 bfr = *reinterpret_cast<const bf16x8*>(&dzT[(lane & 15) * LDM + kk]);
        acc = mfma16x16x32(xf[ks], bfr, acc);
      }
    }
  } else if (aux) {
    bf16x8 ones;
#pragma unroll
    for (int q = 0; q < 8; ++q) ones[q] = (short)0x3f80;  // bf16 1.0
    for (int ks = 0; ks < Mp / 32; ++ks) {
      const int kk = ks * 32 + 8 * (lane >> 4);
      const bf16x8 zT = *reinterpret_cast<const bf16x8*>(&dzT[(lane & 15) * LDM + kk]);
      ab = mfma16x16x32(zT, ones, ab);
      if constexpr (TOP) {
        const bf16x8 h = *reinterpret_cast<const bf16x8*>(&hT[(lane & 15) * LDM + kk]);
        const bf16x8 d = *reinterpret_cast<const bf16x8*>(&dlT[(lane & 15) * LDM + kk]);
        aw = mfma16x16x32(h, d, aw);
        if (lead) ab2 = mfma16x16x32(ones, d, ab2);
      }
    }
  }
  // N > 1 (MdArgs::tx): this tile's gradients -- and (TOP lead) the head's db and the
  // metric slots -- all-reduced with the same tile of the other ranks' launches before
  // the optimizer (common.h tx_tile; payload as mlp_fused.hip's)
  float mval = 0.f;
  if constexpr (TX && !FX) {
    if (TOP && lead && tid < 4) {
      float L = 0.f, Cr = 0.f;
      for (int q = 0; q < NW; ++q) { L += red[0][q]; Cr += red[1][q]; }
      mval = tid == 0 ? L : tid == 2 ? Cr : (float)M;   // {loss sum, n, correct, n}
    }
    float4 v4[2];
    int p4[2] = {0, 0}, n4 = 0, ps = -1;
    float vs = 0.f;
    if (w < NTILE) {
      v4[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
      p4[0] = w * 256 + lane * 4;
      n4 = 1;
      if (TOP && lead && tid < 4) { vs = mval; ps = 9 * 256 + 64 + tid; }
    } else if (aux) {
      v4[0] = make_float4(ab[0], ab[1], ab[2], ab[3]);
      v4[1] = make_float4(aw[0], aw[1], aw[2], aw[3]);
      p4[0] = 7 * 256 + lane * 4;
      p4[1] = 8 * 256 + lane * 4;
      n4 = TOP ? 2 : 1;
      if (TOP && lead && lane < C) { vs = ab2[0]; ps = 9 * 256 + lane; }
    }
    MD_STAMP(5);
    tx_tile(a.tx, a.tx_base + bx * NCH + by, (unsigned)step + 1u, n4, v4, p4, vs, ps,
            a.tx->err);
    MD_STAMP(6);
    if (w < NTILE) {
      acc = (f32x4){v4[0].x, v4[0].y, v4[0].z, v4[0].w};
      if (TOP && lead && tid < 4) mval = vs;
    } else if (aux) {
      ab = (f32x4){v4[0].x, v4[0].y, v4[0].z, v4[0].w};
      if (TOP) aw = (f32x4){v4[1].x, v4[1].y, v4[1].z, v4[1].w};
      if (TOP && lead && lane < C) ab2[0] = vs;
    }
  }
  if constexpr (FX) {
    // FSDP at N > 1 (md_bwd FX): every element's partial goes to the rank owning its row,
    // the owner sums in rank order, applies the sharded AdamW (local state, prefetched at
    // local indices above) and pushes the updated fp32 value to every rank; the
    // replicated b_h and the metric slots are summed by rank T % W and pushed back as
    // sums (every rank updates its own copy).  Then every rank holds the whole updated
    // tile and writes the shadows / hand-offs the next forward reads.
    const TxArgs* X = a.tx;
    const int R = fx_R, W = fx_W;
    const int T = a.tx_base + bx * NCH + by;
    const long pay = __builtin_amdgcn_readfirstlane(X->pay), tiles = __builtin_amdgcn_readfirstlane(X->tiles);
    const unsigned long long tb = (unsigned long long)pay * 4ull;
    const unsigned epoch = (unsigned)step + 1u;
    const long AG = tiles * TX_MAX_RANKS + tiles;   // flag base of the updated-value hand-back
    const int ob = j0 / fx_hpq, orep = T % W;
    const int o_lo = fx_col ? ob : kc0 / fx_rpq, o_hi = fx_col ? ob : (kc0 + KC - 1) / fx_rpq;
    auto owner_of = [&](int q) { return (q >= o_lo && q <= o_hi) || (chunk0 && q == ob) || (lead && q == orep); };
    if (TOP && lead && tid < 4) {
      float L = 0.f, Cr = 0.f;
      for (int q = 0; q < NW; ++q) { L += red[0][q]; Cr += red[1][q]; }
      mval = tid == 0 ? L : tid == 2 ? Cr : (float)M;   // {loss sum, n, correct, n}
    }
    // waves < NTILE: this lane's 4 W elements; aux: lanes ac < C the head's dW rows (TOP),
    // lane ac == C the bias (the column sums are the same in every lane)
    float ev[4] = {0.f, 0.f, 0.f, 0.f};
    int eo[4] = {0, 0, 0, 0}, epos[4] = {0, 0, 0, 0};
    int ne = 0;
    if (w < NTILE) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        ev[e] = acc[e];
        eo[e] = fx_col ? ob : (trow0 + e) / fx_rpq;
        epos[e] = w * 256 + lane * 4 + e;
      }
      ne = 4;
    } else if (aux && ((TOP && ac < C) || ac == C)) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        ev[e] = ac == C ? ab[e] : aw[e];
        eo[e] = ob;
        epos[e] = (ac == C ? 8 * 256 : 7 * 256) + lane * 4 + e;
      }
      ne = 4;
    }
    int rpos = -1;   // replicated scalar of this thread: lead's db_h (aux lanes < C) or a metric slot
    float rv = 0.f;
    if (TOP && lead && aux && lane < C) { rpos = 9 * 256 + lane; rv = ab2[0]; }
    if (TOP && lead && tid < 4) { rpos = 9 * 256 + 64 + tid; rv = mval; }
    // 1. partials to their owners (one uniform resource per candidate owner; a lane whose
    // element belongs elsewhere stores out of range: dropped by the bounds check)
    {
      const int cand[3] = {o_lo, o_hi, ob};
#pragma unroll
      for (int ci = 0; ci < 3; ++ci) {
        const int c = cand[ci];
        if (c == R || (ci >= 1 && c == cand[0]) || (ci == 2 && c == cand[1]) || (ci == 2 && !chunk0)) continue;
        const __amdgpu_buffer_rsrc_t rr = sys_rsrc_u(sgpr_ptr(X->part[c]) + ((long)T * TX_MAX_RANKS + R) * pay, tb);
#pragma unroll
        for (int e = 0; e < 4; ++e) sys_store1(rr, (e < ne && eo[e] == c) ? (long)epos[e] : pay, ev[e]);
      }
    }
    if (rpos >= 0 && orep != R)
      sys_store1(sys_rsrc_u(sgpr_ptr(X->part[orep]) + ((long)T * TX_MAX_RANKS + R) * pay, tb), rpos, rv);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid < W && tid != R && owner_of(tid)) tx_flag_store(X->flag[tid] + (long)T * TX_MAX_RANKS + R, epoch);
    MD_STAMP(5);
    // 2. this rank's owned elements: rank-ordered sums, sharded AdamW, hand-back
    float pnew[4] = {0.f, 0.f, 0.f, 0.f};
    if (owner_of(R)) {
      if (tid < W && tid != R) tx_wait(X->flag[R] + (long)T * TX_MAX_RANKS + tid, epoch, X->timeout, X->err);
      __syncthreads();
      const float* inbox = sgpr_ptr(X->part[R]) + (long)T * TX_MAX_RANKS * pay;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (e >= ne || eo[e] != R) continue;
        float sacc = 0.f;
        for (int q = 0; q < W; ++q) {
          const float x = q == R ? ev[e] : sys_load1(sys_rsrc_u(inbox + (long)q * pay, tb), epos[e]);
          sacc = q == 0 ? x : sacc + x;
        }
        ev[e] = sacc;
      }
      if (rpos >= 0 && orep == R) {
        float sacc = 0.f;
        for (int q = 0; q < W; ++q) {
          const float x = q == R ? rv : sys_load1(sys_rsrc_u(inbox + (long)q * pay, tb), rpos);
          sacc = q == 0 ? x : sacc + x;
        }
        rv = sacc;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (e >= ne || eo[e] != R) continue;
        float tp, tm, tv;
        if (w < NTILE) {
          const long li = fx_col ? (long)(trow0 + e) * fx_hpq + (tcol - R * fx_hpq)
                                 : (long)(trow0 + e - R * fx_rpq) * N + tcol;
          md_adam(op[e], om[e], ov[e], ev[e], ak, &tp, &tm, &tv);
          a.pW[li] = tp; a.mW[li] = tm; a.vW[li] = tv;
        } else {
          const int lr_ = j0 + (lane >> 4) * 4 + e - R * fx_hpq;
          if (ac == C) {
            md_adam(bp[e], bm[e], bvv[e], ev[e], ak, &tp, &tm, &tv);
            a.pb[lr_] = tp; a.mb[lr_] = tm; a.vb[lr_] = tv;
          } else {
            const long li = (long)lr_ * C + ac;
            md_adam(op[e], om[e], ov[e], ev[e], ak, &tp, &tm, &tv);
            a.pWh[li] = tp; a.mWh[li] = tm; a.vWh[li] = tv;
          }
        }
        pnew[e] = tp;
      }
      for (int q = 0; q < W; ++q) {
        if (q == R) continue;
        const __amdgpu_buffer_rsrc_t dst = sys_rsrc_u(sgpr_ptr(X->red[q]) + (long)T * pay, tb);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (e < ne && eo[e] == R) sys_store1(dst, epos[e], pnew[e]);
        if (rpos >= 0 && orep == R) sys_store1(dst, rpos, rv);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid < W && tid != R) tx_flag_store(X->flag[tid] + AG + (long)T * TX_MAX_RANKS + R, epoch);
    }
    // 3. the other owners' updated values
    if (tid < W && tid != R && owner_of(tid))
      tx_wait(X->flag[R] + AG + (long)T * TX_MAX_RANKS + tid, epoch, X->timeout, X->err);
    __syncthreads();
    {
      const __amdgpu_buffer_rsrc_t src = sys_rsrc_u(sgpr_ptr(X->red[R]) + (long)T * pay, tb);
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (e < ne && eo[e] != R) pnew[e] = sys_load1(src, epos[e]);
      if (rpos >= 0 && orep != R) rv = sys_load1(src, rpos);
    }
    if (TOP && lead && tid < 4) mval = rv;
    MD_STAMP(6);
    // 4. the whole updated tile: the next step's row-major shadow, W^T copy and (layer 0)
    // the run-ahead forward's LDS image; bias shadow / hand-off; head shadow; b_h
    // (replicated) updated by every rank from the summed gradient
    const int par_s = __builtin_amdgcn_readfirstlane(par);
    if (w < NTILE) {
      bf16_t* Wsn = const_cast<bf16_t*>(par_s ? a.Ws0 : a.Ws1);
      const __amdgpu_buffer_rsrc_t wsn_r = __builtin_amdgcn_make_buffer_rsrc(Wsn, (short)0, 0x7fffffff, 0x00020000);
      unsigned wtp[2] = {0u, 0u};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bf16_t pb = f2bf(pnew[e]);
        const long idx = (long)(trow0 + e) * N + tcol;
        if (a.wt & 2) __builtin_amdgcn_raw_buffer_store_b16((unsigned short)pb, wsn_r, (int)(idx * 2), 0, 16);
        else Wsn[idx] = pb;
        wtp[e >> 1] |= (unsigned)pb << (16 * (e & 1));
      }
      if (a.WTout) {
        bf16_t* const wto = a.WTout + (long)tcol * a.ldwt + trow0;
        __hip_atomic_store((__attribute__((address_space(1))) unsigned long long*)wto,
                           (unsigned long long)wtp[0] | ((unsigned long long)wtp[1] << 32), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
      if constexpr (AHEAD)
        *reinterpret_cast<uint2*>(&w1n[(lane & 15) * LDW1 + (trow0 - kc0)]) = make_uint2(wtp[0], wtp[1]);
    } else if (aux) {
      bf16_t* Whn = const_cast<bf16_t*>(par_s ? a.Wh0 : a.Wh1);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int j = j0 + (lane >> 4) * 4 + e;
        if (TOP && ac < C) Whn[(long)j * C + ac] = f2bf(pnew[e]);
        if (ac == C) {
          a.sb[j] = f2bf(pnew[e]);
          if constexpr (AHEAD) a.hand[j] = pnew[e];   // the next forward's bias (same XCD: L2 hand-off)
        }
      }
      if (TOP && lead && lane < C) a.sbh[lane] = f2bf(md_adam(qp, qm, qv, rv, ak, a.pbh + lane, a.mbh + lane, a.vbh + lane));
    }
  } else {
    // the step parity as a scalar for the parity-selected store resources (the step was the
    // first load of the launch and is long back; per lane it made them waterfall loops)
    const int par_s = __builtin_amdgcn_readfirstlane(par);
    if (w < NTILE) {
      bf16_t* Wsn = const_cast<bf16_t*>(par_s ? a.Ws0 : a.Ws1);   // next step's parity of the row-major shadow
      const __amdgpu_buffer_rsrc_t wsn_r = __builtin_amdgcn_make_buffer_rsrc(Wsn, (short)0, 0x7fffffff, 0x00020000);
      unsigned wtp[2] = {0u, 0u};
  #pragma unroll
      for (int e = 0; e < 4; ++e) {
        const long idx = (long)(trow0 + e) * N + tcol;
        if (a.fuse_opt) {
          float tp, tm, tv;
          const bf16_t pb = f2bf(md_adam(op[e], om[e], ov[e], acc[e], ak, &tp, &tm, &tv));
          if (a.wt & 1) {
            md_st(a.pW + idx, tp); md_st(a.mW + idx, tm); md_st(a.vW + idx, tv);
          } else {
            a.pW[idx] = tp; a.mW[idx] = tm; a.vW[idx] = tv;
          }
          if (a.wt & 2)   // the next step's bf16 row-major shadow, write-through too
            __builtin_amdgcn_raw_buffer_store_b16((unsigned short)pb, wsn_r, (int)(idx * 2), 0, 16);
          else
            Wsn[idx] = pb;
          wtp[e >> 1] |= (unsigned)pb << (16 * (e & 1));
        } else if (a.smap) {
          stage_store(a.smap, par, 0, trow0 + e, tcol, acc[e]);
        } else {
          a.gW[goff + idx] = (a.accumulate ? op[e] : 0.f) + acc[e];   // mode 0 loaded the old grad into op
        }
      }
      if (a.fuse_opt && a.WTout) {
        bf16_t* const wto = a.WTout + (long)tcol * a.ldwt + trow0;
        if (a.wt & 1)
          __hip_atomic_store((__attribute__((address_space(1))) unsigned long long*)wto,
                             (unsigned long long)wtp[0] | ((unsigned long long)wtp[1] << 32), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        else
          *reinterpret_cast<uint2*>(wto) = make_uint2(wtp[0], wtp[1]);
      }
      if constexpr (AHEAD)
        *reinterpret_cast<uint2*>(&w1n[(lane & 15) * LDW1 + (trow0 - kc0)]) = make_uint2(wtp[0], wtp[1]);
    } else if (aux) {
      bf16_t* Whn = const_cast<bf16_t*>(par_s ? a.Wh0 : a.Wh1);
  #pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = (lane >> 4) * 4 + e;
        if (TOP && ac < C) {
          const long g = (long)(j0 + n) * C + ac;
          if (a.fuse_opt) Whn[g] = f2bf(md_adam(op[e], om[e], ov[e], aw[e], ak, a.pWh + g, a.mWh + g, a.vWh + g));
          else if (a.smap) stage_store(a.smap, par, 2, j0 + n, ac, aw[e]);
          else a.gWh[goff + g] = (a.accumulate ? op[e] : 0.f) + aw[e];
        }
        if (ac == 0) {
          const int j = j0 + n;
          if (a.fuse_opt) {
            const float pn = md_adam(bp[e], bm[e], bvv[e], ab[e], ak, a.pb + j, a.mb + j, a.vb + j);
            a.sb[j] = f2bf(pn);
            if constexpr (AHEAD) a.hand[j] = pn;   // the next forward's bias (same XCD: L2 hand-off)
          } else if (a.smap) {
            stage_store(a.smap, par, 1, j, 0, ab[e]);
          } else {
            a.gb[goff + j] = (a.accumulate ? bp[e] : 0.f) + ab[e];
          }
        }
      }
      if (TOP && lead && lane < C) {
        if (a.fuse_opt) a.sbh[lane] = f2bf(md_adam(qp, qm, qv, ab2[0], ak, a.pbh + lane, a.mbh + lane, a.vbh + lane));
        else if (a.smap) stage_store(a.smap, par, 3, lane, 0, ab2[0]);
        else a.gbh[goff + lane] = (a.accumulate ? qp : 0.f) + ab2[0];
      }
    }
  }
  MD_STAMP(3);
  if (TOP && lead) {
    __syncthreads();
    if (TX) {   // the all-reduced slots, one per thread
      if (tid < 4 && a.fuse_opt && a.running) a.running[tid] += mval;
    } else if (tid == 0) {
      float L = 0.f, Cr = 0.f;
      for (int q = 0; q < NW; ++q) { L += red[0][q]; Cr += red[1][q]; }
      if (a.fuse_opt && a.running) {
        a.running[0] += L; a.running[1] += (float)M; a.running[2] += Cr; a.running[3] += (float)M;
      } else if (a.smap) {
        stage_store(a.smap, par, 4, 0, 0, L); stage_store(a.smap, par, 4, 1, 0, (float)M);
        stage_store(a.smap, par, 4, 2, 0, Cr); stage_store(a.smap, par, 4, 3, 0, (float)M);
      } else if (a.mslot) {
        const float k = a.accumulate ? 1.f : 0.f;
        float* ms = a.mslot + goff;
        ms[0] = k * ms[0] + L; ms[1] = k * ms[1] + (float)M;
        ms[2] = k * ms[2] + Cr; ms[3] = k * ms[3] + (float)M;
      }
    }
  }
  unsigned launch_no = 0u;
  if constexpr (AHEAD) {
    // ---- 5. step t+1's layer-0 forward (see mlp_fused.hip mlp2_bwd AHEAD): partial
    // Z_0 of (chunk, blk) from the W_0' tile just produced, column-block barrier in the
    // XCD's L2, then each of the NCH workgroups finishes a share of the rows
    __syncthreads();   // w1n complete, hand-off stored
    unsigned tile_seen = 0u;
    if (tid == 0) {
      launch_no = a.ztick[2];
      const int tpx = (N / 16) * NCH / 8, t = bx * NCH + by;
      tile_seen = __hip_atomic_fetch_add((gu32_md*)(a.ztick + 32 * (1 + N / 16) + 32 * ((tpx + 31) / 32) * (t / tpx) + t % tpx),
                                         1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      if (ks * 32 < KC) {
        const bf16x8 bw = *reinterpret_cast<const bf16x8*>(&w1n[(lane & 15) * LDW1 + ks * 32 + 8 * (lane >> 4)]);
        z = mfma16x16x32(xa[ks], bw, z);
      }
    }
    float* const zb = a.zslab + (long)bx * NCH * (MPM / 4) * 64;
    *reinterpret_cast<u32x4*>(zb + ((long)by * (MPM / 4) + w * 4 + (lane >> 4)) * 64 + (lane & 15) * 4) =
        (u32x4){__float_as_uint(z[0]), __float_as_uint(z[1]), __float_as_uint(z[2]), __float_as_uint(z[3])};
    // step t+1's dropout bits of this thread's epilogue element, while the store drains
    if (a.keep < 1.f && eg < g_hi && eg * 4 < M) {
      const int sn = step + 1;
      int lrow = eg * 4, Mg = M;
      unsigned long long off = a.offset + ((unsigned long long)(unsigned)(a.step_mul > 1 ? sn * a.step_mul : sn) << 32);
      if (a.mb_rows > 0) {   // per-microbatch streams, as md_fwd draws them
        const int mi = (eg * 4) / a.mb_rows;
        lrow = eg * 4 - mi * a.mb_rows;
        Mg = a.mb_rows;
        off += (unsigned long long)mi * a.mb_stride;
      }
      dbn = dropout_bits(a.seed, off, dropout_group(0, lrow, j0 + gn, Mg, N));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      unsigned* cnt = a.ztick + 32 * (1 + bx);
      __hip_atomic_fetch_add((gu32_md*)cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      const unsigned target = (unsigned)NCH * (launch_no + 1u);
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      const __amdgpu_buffer_rsrc_t cr = __builtin_amdgcn_make_buffer_rsrc(cnt, (short)0, 4, 0x00020000);
      while ((int)((unsigned)__builtin_amdgcn_raw_buffer_load_b32(cr, 0, 0, 16) - target) < 0) {
        if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > 2000000ll) {   // 20 ms
          atomicOr(a.ztick + 1, 2u);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        asm volatile("" ::: "memory");
      }
      if (tile_seen != launch_no) atomicOr(a.ztick + 1, 1u);
    }
    __syncthreads();
    // ---- 6. layer 0's forward epilogue of step t+1, one element per thread
    const int ng = g_hi - g_lo;
    const __amdgpu_buffer_rsrc_t zr = __builtin_amdgcn_make_buffer_rsrc(zb, (short)0, NCH * (MPM / 4) * 64 * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t hr = __builtin_amdgcn_make_buffer_rsrc(a.hand, (short)0, N * 4, 0x00020000);
    const int egc = min(eg, g_hi - 1);
    float zp[NCH];
#pragma unroll
    for (int q = 0; q < NCH; ++q)
      zp[q] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                            zr, (int)((((long)q * (MPM / 4) + egc) * 64 + gn * 4 + ee) * 4), 0, 16));
    const float bv = round_bf(__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(hr, (j0 + gn) * 4, 0, 16)));
    if (tid < 64 * ng) {
      const int row = eg * 4 + ee;
      if (row < M) {
        float v = bv;   // + the NCH chunk partials in chunk order
#pragma unroll
        for (int q = 0; q < NCH; ++q) v += zp[q];
        const float zz = bf2f(f2bf(v));           // Z_0 as the bf16 Dense output
        const float ez = __expf(-zz);
        const float sg = 1.0f / (1.0f + ez);
        float hvn = zz * sg;                       // act_fwd(ACT_SILU), as md_fwd
        float gd = sg * (1.0f + zz * (1.0f - sg));  // act_grad(ACT_SILU)
        if (a.keep < 1.f) {
          const bool kp = keep_word(dbn, ee, a.keep);
          hvn = kp ? hvn / a.keep : 0.f;
          gd = kp ? gd / a.keep : 0.f;
        }
        a.Hout[(long)row * N + j0 + gn] = f2bf(hvn);
        a.G[((long)eg * N + j0 + gn) * 4 + ee] = gd;
      }
    }
  }
  if (a.advance_step) {
    __syncthreads();
    if (tid == 0) {
      const unsigned t = atomicAdd(a.ticket, 1u);
      if (t == gridDim.x * gridDim.y - 1) {
        a.step[0] = step + 1;
        if constexpr (AHEAD) a.ztick[2] = launch_no + 1u;   // every workgroup has read it (ticket)
        __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

}  // namespace jdt
using namespace jdt;

int xcd_tiles_enabled();   // mlp_fused.hip (JDT_XCD_TILES)
int xcd_roundrobin_ok(int G);   // mlp_fused.hip (XCD dispatch probe)

JDT_API int jdt_md_args_size() { return (int)sizeof(MdArgs); }

// 1 if the run-ahead layer-0 backward fits (its column barrier needs every workgroup resident)
JDT_API int jdt_md_ahead_ok(int M) {
  if (M <= 0 || M > MD_MPM) return 0;
  if (!xcd_roundrobin_ok((512 / 16) * (784 / 112))) return 0;
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, md_bwd_kernel<784, false, 10, 112, 512, true, false, true>,
                                                   MD_NT, 0) != hipSuccess)
    return 0;
  return (512 / 16) * (784 / 112) <= cus * per ? 1 : 0;
}

// 1 if the dZ split (MdArgs::dzs) fits: its per-block arrival counter needs every
// workgroup of the !TOP backward grids resident at once
JDT_API int jdt_md_dzs_ok(int M) {
  if (M <= 0 || M > MD_MPM) return 0;
  int dev = 0, cus = 0, p1 = 0, p2 = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&p1, md_bwd_kernel<512, false, 10, 64, 512, true>, MD_NT, 0) !=
          hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&p2, md_bwd_kernel<784, false, 10, 112, 512, true>, MD_NT, 0) !=
          hipSuccess)
    return 0;
  return (512 / 16) * (512 / 64) <= cus * p1 && (512 / 16) * (784 / 112) <= cus * p2 ? 1 : 0;
}

// 1 if md_fwd2_kernel's row-block counters can work for M rows: every workgroup of its
// (ceil(M / 16), 32) grid resident at once
JDT_API int jdt_md_fwd2_ok(int M) {
  if (M <= 0 || M > MD_MPM) return 0;
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, md_fwd2_kernel, MD_NT, 0) != hipSuccess)
    return 0;
  return ((M + 15) / 16) * 32 <= cus * per ? 1 : 0;
}

// layers i (a1) and i + 1 (a2, with the head) of a deep MLP's forward in one launch
// (md_fwd2_kernel): both 512 -> 512, the W^T copies present (fused-optimizer mode)
JDT_API int jdt_md_fwd2(const MdArgs* a1, const MdArgs* a2, unsigned* rowc, void* stream) {
  const MdArgs& x = *a1;
  const MdArgs& y = *a2;
  if (x.K != 512 || y.K != 512 || x.N != 512 || y.N != 512 || x.M != y.M || x.M <= 0 || x.M > MD_MPM || y.C != 10 ||
      !x.WT || !y.WT || !rowc || x.Hout != y.X)
    return -3;
  if (x.mb_rows < 0 || (x.mb_rows && (x.mb_rows % 4 || x.M % x.mb_rows)) || y.mb_rows < 0 ||
      (y.mb_rows && (y.mb_rows % 4 || y.M % y.mb_rows)))
    return -2;
  hipLaunchKernelGGL(md_fwd2_kernel, dim3((x.M + 15) / 16, x.N / 16), dim3(MD_NT), 0, static_cast<hipStream_t>(stream),
                     x, y, rowc);
  return HIP_LAUNCH_CHECK();
}

// phase 0: forward of one hidden layer (head = 1: + head logits); phase 1: backward
// (head = 1: TOP layer, CE through the head; head = 2: pipeline-stage boundary,
// dZ from the next stage's dH).  Instantiated for the tutorial
// shapes: K in {784 (fp32 data), 512}, N = NN = 512, C = 10, M <= 128.
// 1 if the deep engine's N > 1 step with the in-kernel tile exchange can run here with
// `nshare` ranks' grids on this GPU: every exchanging backward launch of every sharing
// rank resident at once (as jdt_mlp2_ahead_tx_ok).
template <bool FX>
static int md_tx_fits(int M, int nshare) {
  if (M <= 0 || M > MD_MPM || nshare < 1) return 0;
  int dev = 0, cus = 0, p0 = 0, p1 = 0, p2 = 0;
  const bool sh = nshare > 1;   // the launcher's variant choice (MdArgs::tx_shared)
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &p0,
          sh ? (const void*)md_bwd_kernel<784, false, 10, 112, 512, true, false, true, true, 4, FX>
             : (const void*)md_bwd_kernel<784, false, 10, 112, 512, true, false, true, true, 1, FX>,
          MD_NT, 0) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&p1, md_bwd_kernel<512, true, 10, 64, 512, true, false, false, true, 1, FX>,
                                                   MD_NT, 0) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &p2,
          sh ? (const void*)md_bwd_kernel<512, false, 10, 64, 512, true, false, false, true, 4, FX>
             : (const void*)md_bwd_kernel<512, false, 10, 64, 512, true, false, false, true, 1, FX>,
          MD_NT, 0) != hipSuccess)
    return 0;
  const long cap = (long)cus * (p0 < p1 ? (p0 < p2 ? p0 : p2) : (p1 < p2 ? p1 : p2));
  return (long)nshare * (512 / 16) * (512 / 64) <= cap ? 1 : 0;
}
JDT_API int jdt_md_tx_ok(int M, int nshare) { return md_tx_fits<false>(M, nshare); }
// the same for the FSDP form (md_bwd FX, MdArgs::tx_fsdp)
JDT_API int jdt_md_fx_ok(int M, int nshare) { return md_tx_fits<true>(M, nshare); }

JDT_API int jdt_md_layer(const MdArgs* args, int phase, int head, void* stream) {
  const MdArgs& a = *args;
  if (a.N != 512 || a.M <= 0 || a.M > MD_MPM || (a.K != 784 && a.K != 512) || (head == 1 && a.C != 10)) return -3;
  if (phase == 0 && head == 2) return -2;
  if (a.mb_rows < 0 || (a.mb_rows && (a.mb_rows % 4 || a.M % a.mb_rows))) return -2;
  if (a.dzs && (phase == 0 || head || !a.dzx || !a.dzc)) return -2;   // dZ split: !TOP, !BND backward only
  hipStream_t st = static_cast<hipStream_t>(stream);
  const dim3 blk(MD_NT);
  if (phase == 2) {
    // run-ahead layer-0 backward (+ layer 0's forward of the next step)
    if (a.K != 784 || head || !a.fuse_opt || !a.WTout || !a.XR || !a.zslab || !a.ztick || !a.hand ||
        !a.advance_step || a.det_logits)
      return -3;
    if (a.tx && a.tx_fsdp && a.tx_shared)
      hipLaunchKernelGGL((md_bwd_kernel<784, false, 10, 112, 512, true, false, true, true, 4, true>),
                         dim3(a.N / 16, 784 / 112), blk, 0, st, a);
    else if (a.tx && a.tx_fsdp)
      hipLaunchKernelGGL((md_bwd_kernel<784, false, 10, 112, 512, true, false, true, true, 1, true>),
                         dim3(a.N / 16, 784 / 112), blk, 0, st, a);
    else if (a.tx && a.tx_shared)
      hipLaunchKernelGGL((md_bwd_kernel<784, false, 10, 112, 512, true, false, true, true, 4>),
                         dim3(a.N / 16, 784 / 112), blk, 0, st, a);
    else if (a.tx)
      hipLaunchKernelGGL((md_bwd_kernel<784, false, 10, 112, 512, true, false, true, true>), dim3(a.N / 16, 784 / 112),
                         blk, 0, st, a);
    else
      hipLaunchKernelGGL((md_bwd_kernel<784, false, 10, 112, 512, true, false, true>), dim3(a.N / 16, 784 / 112), blk,
                         0, st, a);
    return HIP_LAUNCH_CHECK();
  }
  if (a.tx && phase == 1) {
    // N > 1 hidden layers >= 1 with the in-kernel tile exchange (layer 0 runs ahead)
    if (a.K != 512 || head == 2 || a.dzs || !a.fuse_opt) return -3;
    const dim3 g(a.N / 16, 512 / 64);
    if (a.tx_fsdp) {
      if (head)
        hipLaunchKernelGGL((md_bwd_kernel<512, true, 10, 64, 512, true, false, false, true, 1, true>), g, blk, 0, st, a);
      else if (a.tx_shared)
        hipLaunchKernelGGL((md_bwd_kernel<512, false, 10, 64, 512, true, false, false, true, 4, true>), g, blk, 0, st, a);
      else
        hipLaunchKernelGGL((md_bwd_kernel<512, false, 10, 64, 512, true, false, false, true, 1, true>), g, blk, 0, st, a);
      return HIP_LAUNCH_CHECK();
    }
    if (head) hipLaunchKernelGGL((md_bwd_kernel<512, true, 10, 64, 512, true, false, false, true>), g, blk, 0, st, a);
    else if (a.tx_shared)
      hipLaunchKernelGGL((md_bwd_kernel<512, false, 10, 64, 512, true, false, false, true, 4>), g, blk, 0, st, a);
    else hipLaunchKernelGGL((md_bwd_kernel<512, false, 10, 64, 512, true, false, false, true>), g, blk, 0, st, a);
    return HIP_LAUNCH_CHECK();
  }
  if (phase == 0) {
    // 16-row blocks: twice the workgroups, half the input bytes each (as mlp2_fwd)
    const dim3 grid((a.M + 15) / 16, a.N / 16);
    const bool d = a.WT != nullptr;
    const bool xf = xcd_tiles_enabled() == 1;
    if (a.K == 784 && head) {
      // a one-hidden-layer MLP (the 2-layer tutorial classifier) per microbatch
      if (d) { if (xf) hipLaunchKernelGGL((md_fwd_kernel<784, true, 112, true, 10, 16, true, true>), grid, blk, 0, st, a); else hipLaunchKernelGGL((md_fwd_kernel<784, true, 112, true, 10, 16, true, false>), grid, blk, 0, st, a); }
      else { if (xf) hipLaunchKernelGGL((md_fwd_kernel<784, true, 112, true, 10, 16, false, true>), grid, blk, 0, st, a); else hipLaunchKernelGGL((md_fwd_kernel<784, true, 112, true, 10, 16, false, false>), grid, blk, 0, st, a); }
    } else if (a.K == 784) {
      if (d) { if (xf) hipLaunchKernelGGL((md_fwd_kernel<784, true, 112, false, 10, 16, true, true>), grid, blk, 0, st, a); else hipLaunchKernelGGL((md_fwd_kernel<784, true, 112, false, 10, 16, true, false>), grid, blk, 0, st, a); }
      else { if (xf) hipLaunchKernelGGL((md_fwd_kernel<784, true, 112, false, 10, 16, false, true>), grid, blk, 0, st, a); else hipLaunchKernelGGL((md_fwd_kernel<784, true, 112, false, 10, 16, false, false>), grid, blk, 0, st, a); }
    } else if (head) {
      if (d) { if (xf) hipLaunchKernelGGL((md_fwd_kernel<512, false, 16, true, 10, 16, true, true>), grid, blk, 0, st, a); else hipLaunchKernelGGL((md_fwd_kernel<512, false, 16, true, 10, 16, true, false>), grid, blk, 0, st, a); }
      else { if (xf) hipLaunchKernelGGL((md_fwd_kernel<512, false, 16, true, 10, 16, false, true>), grid, blk, 0, st, a); else hipLaunchKernelGGL((md_fwd_kernel<512, false, 16, true, 10, 16, false, false>), grid, blk, 0, st, a); }
    } else {
      if (d) { if (xf) hipLaunchKernelGGL((md_fwd_kernel<512, false, 16, false, 10, 16, true, true>), grid, blk, 0, st, a); else hipLaunchKernelGGL((md_fwd_kernel<512, false, 16, false, 10, 16, true, false>), grid, blk, 0, st, a); }
      else { if (xf) hipLaunchKernelGGL((md_fwd_kernel<512, false, 16, false, 10, 16, false, true>), grid, blk, 0, st, a); else hipLaunchKernelGGL((md_fwd_kernel<512, false, 16, false, 10, 16, false, false>), grid, blk, 0, st, a); }
    }
  } else if (head == 2) {
    // pipeline-stage boundary: dZ_i = dH * G_i
    if (!a.dH) return -2;
    const bool x = xcd_tiles_enabled() != 0;
    if (a.K == 784) {
      const dim3 g(a.N / 16, 784 / 112);
      if (x) hipLaunchKernelGGL((md_bwd_kernel<784, false, 10, 112, 512, true, true>), g, blk, 0, st, a);
      else hipLaunchKernelGGL((md_bwd_kernel<784, false, 10, 112, 512, false, true>), g, blk, 0, st, a);
    } else {
      const dim3 g(a.N / 16, 512 / 64);
      if (x) hipLaunchKernelGGL((md_bwd_kernel<512, false, 10, 64, 512, true, true>), g, blk, 0, st, a);
      else hipLaunchKernelGGL((md_bwd_kernel<512, false, 10, 64, 512, false, true>), g, blk, 0, st, a);
    }
  } else {
    const bool x = xcd_tiles_enabled() != 0;
    if (a.K == 784) {
      const dim3 g(a.N / 16, 784 / 112);
      if (head) {  // TOP layer with a 784-wide input: the 2-layer classifier
        if (x) hipLaunchKernelGGL((md_bwd_kernel<784, true, 10, 112, 512, true>), g, blk, 0, st, a);
        else hipLaunchKernelGGL((md_bwd_kernel<784, true, 10, 112, 512, false>), g, blk, 0, st, a);
      } else {
        if (x) hipLaunchKernelGGL((md_bwd_kernel<784, false, 10, 112, 512, true>), g, blk, 0, st, a);
        else hipLaunchKernelGGL((md_bwd_kernel<784, false, 10, 112, 512, false>), g, blk, 0, st, a);
      }
    } else if (head) {
      const dim3 g(a.N / 16, 512 / 64);
      if (x) hipLaunchKernelGGL((md_bwd_kernel<512, true, 10, 64, 512, true>), g, blk, 0, st, a);
      else hipLaunchKernelGGL((md_bwd_kernel<512, true, 10, 64, 512, false>), g, blk, 0, st, a);
    } else {
      const dim3 g(a.N / 16, 512 / 64);
      if (x) hipLaunchKernelGGL((md_bwd_kernel<512, false, 10, 64, 512, true>), g, blk, 0, st, a);
      else hipLaunchKernelGGL((md_bwd_kernel<512, false, 10, 64, 512, false>), g, blk, 0, st, a);
    }
  }
  return HIP_LAUNCH_CHECK();
}
