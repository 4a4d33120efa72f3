// Shared device helpers for the gfx950 (CDNA4 / MI355X) kernel library.
//
// Everything here is written for 64-lane wavefronts and the gfx950 MFMA
// intrinsics; there is no other target.  Host code reaches the kernels through
// the extern "C" launchers in each .hip file (loaded with ctypes from
// ops/_lib.py), always on the caller's HIP stream so that the whole training
// step can be captured into one hipGraph.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define JDT_API extern "C" __attribute__((visibility("default")))

namespace jdt {

typedef uint16_t bf16_t;  // raw bf16 bits
typedef __attribute__((ext_vector_type(8))) short bf16x8;  // MFMA A/B fragment
typedef __attribute__((ext_vector_type(4))) float f32x4;   // 16x16 MFMA C/D
typedef __attribute__((ext_vector_type(16))) float f32x16; // 32x32 MFMA C/D
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

constexpr int WAVE = 64;

// ---------------------------------------------------------------- bf16 <-> f32
__device__ __forceinline__ float bf2f(bf16_t h) {
  return __uint_as_float(((uint32_t)h) << 16);
}
// round-to-nearest-even.  gfx950 has a hardware RNE convert (v_cvt_pk_bf16_f32,
// two values per instruction); the __bf16 cast lowers to it, replacing the
// 5-6 VALU ops of the integer rounding trick (PMC: the fused MLP kernels were
// VALU-bound on conversions).
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}
__device__ __forceinline__ float round_bf(float f) { return bf2f(f2bf(f)); }

// ---------------------------------------------------------------- FSDP staged gradient bucket
// A producer kernel of the FSDP step (mlp2_bwd / md_bwd mode 0) writes each full-layout
// gradient element straight into this rank's xGMI data buffer, in the packed layout of
// the fused FSDP collective (comm/csrc/xgmi.hip xg_fsdp_kernel, staged): peer-part q of
// leaf k at q * slice + off_k (+ the element's index within the part), in the half of
// the optimizer step's parity -- so the collective skips its staging copy.
struct StageLeaf {
  long off;    // packed offset (words) of this leaf's part within a peer slot
  int dim;     // 0: row shards of `per` rows; 1: column shards of `per` columns;
               // 2: replicated leaf / metric slots (the whole leaf in every peer slot)
  int per;
  int cols;    // row length of the full leaf (1 for a vector)
  int pad;
};
struct StageMap {
  float* base;   // this rank's IPC data buffer, half 0
  long half;     // floats from half 0 to half 1
  long slice;    // floats per peer slot
  int W;         // ranks
  int nleaf;
  StageLeaf leaf[5];   // the producer's outputs: [0] W, [1] b, [2] head W, [3] head b, [4] metrics
};

__device__ __forceinline__ void stage_store(const StageMap* m, int par, int leaf, int row, int col, float v) {
  const StageLeaf L = m->leaf[leaf];
  // a global (not flat) pointer: a flat store also counts in lgkmcnt, so every later LDS
  // wait of the producer would wait for these stores' write acknowledgements too
  __attribute__((address_space(1))) float* b =
      (__attribute__((address_space(1))) float*)(m->base + (long)par * m->half + L.off);
  if (L.dim == 2) {
    for (int q = 0; q < m->W; ++q) b[(long)q * m->slice + (long)row * L.cols + col] = v;
    return;
  }
  const int q = (L.dim == 0 ? row : col) / L.per;
  const long jj = L.dim == 0 ? (long)(row - q * L.per) * L.cols + col : (long)row * L.per + (col - q * L.per);
  b[(long)q * m->slice + jj] = v;
}

// ---------------------------------------------------------------- reductions
// Whole-wave sum through DPP lane moves (no LDS): quad_perm swaps (xor 1, xor 2),
// row_half_mirror and row_mirror leave every 16-lane row uniform, then the four
// row values are read into SGPRs.  The ds_bpermute butterfly of wave_sum costs
// one LDS round trip (and an lgkmcnt wait) per step: 6 dependent round trips.
// The result is identical in every lane (fixed order).
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);  // row_half_mirror
  v += dpp_mov<0x140>(v);  // row_mirror
  const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
  const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 16));
  const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32));
  const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 48));
  return (r0 + r1) + (r2 + r3);
}

// 8 bf16 sums a + b (fp32 add, round to nearest even): the token + position embedding,
// shared by embed_fwd_kernel and the embedding-fused LayerNorm so both give the same bits
__device__ __forceinline__ u32x4 bf16x8_add(u32x4 a, u32x4 b) {
  u32x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float lo = bf2f((bf16_t)(a[j] & 0xffff)) + bf2f((bf16_t)(b[j] & 0xffff));
    const float hi = bf2f((bf16_t)(a[j] >> 16)) + bf2f((bf16_t)(b[j] >> 16));
    o[j] = (unsigned)f2bf(lo) | ((unsigned)f2bf(hi) << 16);
  }
  return o;
}

__device__ __forceinline__ float wave_max_dpp(float v) {
  v = fmaxf(v, dpp_mov<0xB1>(v));
  v = fmaxf(v, dpp_mov<0x4E>(v));
  v = fmaxf(v, dpp_mov<0x141>(v));
  v = fmaxf(v, dpp_mov<0x140>(v));
  const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
  const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 16));
  const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32));
  const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 48));
  return fmaxf(fmaxf(r0, r1), fmaxf(r2, r3));
}
template <int CTRL>
__device__ __forceinline__ int dpp_movi(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false); }
__device__ __forceinline__ int wave_min_dpp(int v) {
  v = min(v, dpp_movi<0xB1>(v));
  v = min(v, dpp_movi<0x4E>(v));
  v = min(v, dpp_movi<0x141>(v));
  v = min(v, dpp_movi<0x140>(v));
  return min(min(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
             min(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, WAVE));
  return v;
}

// ---------------------------------------------------------------- LayerNorm arithmetic
// Shared by ln_fwd_kernel and the LN-prologue GEMM (gemm_ln_kernel) with explicit
// rounding intrinsics, so hipcc's default FMA contraction cannot make the two
// produce different bf16 values for the same row.
__device__ __forceinline__ float ln_sq_acc(float q, float x, float mean) {
  const float t = __fsub_rn(x, mean);
  return __fmaf_rn(t, t, q);
}
__device__ __forceinline__ float ln_norm(float x, float mean, float rstd, float g, float b) {
  return __fmaf_rn(__fmul_rn(__fsub_rn(x, mean), rstd), g, b);
}

// ---------------------------------------------------------------- Philox4x32-10
// Counter-based RNG: the dropout mask of element `idx` under stream (seed,
// offset) is a pure function, so the backward pass regenerates it instead of
// storing a mask tensor.  `offset` folds in (step, minibatch,
// rank) exactly like jax.random.fold_in does for the reference's dropout key
// (data_paral.py:28-34, 178).
__device__ __forceinline__ u32x4 philox4x32(uint64_t seed, uint64_t ctr_lo, uint64_t ctr_hi) {
  uint32_t c0 = (uint32_t)ctr_lo, c1 = (uint32_t)(ctr_lo >> 32);
  uint32_t c2 = (uint32_t)ctr_hi, c3 = (uint32_t)(ctr_hi >> 32);
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  u32x4 out; out.x = c0; out.y = c1; out.z = c2; out.w = c3;
  return out;
}
// Dropout mask of element (z, r, c) of a [.., M, N] activation: one Philox call
// yields the decisions of the 4-row group (r & ~3 .. r | 3) at column c -- word
// (r & 3) of philox(seed, counter = (z * ceil(M/4) + r/4) * N + c, offset).  Every
// kernel that touches the mask (GEMM epilogues, act_bwd, the fused step kernels)
// owns whole 4-row groups, so the 10-round Philox is paid once per 4 elements.
__device__ __forceinline__ uint64_t dropout_group(int z, int r, int c, int M, int N) {
  return ((uint64_t)z * (uint64_t)((M + 3) >> 2) + (uint64_t)(r >> 2)) * (uint64_t)N + (uint64_t)c;
}
__device__ __forceinline__ u32x4 dropout_bits(uint64_t seed, uint64_t offset, uint64_t group) {
  return philox4x32(seed, group, offset);
}
__device__ __forceinline__ bool keep_word(const u32x4& b, int w, float keep_prob) {
  const unsigned x = w == 0 ? b.x : (w == 1 ? b.y : (w == 2 ? b.z : b.w));
  return (float)(x >> 8) * (1.0f / 16777216.0f) < keep_prob;
}

// ---------------------------------------------------------------- activations
enum Act : int { ACT_NONE = 0, ACT_SILU = 1, ACT_GELU = 2, ACT_RELU = 3 };

// tanh through one exp and one reciprocal: tanh(u) = 1 - 2 / (exp(2u) + 1).  libm's
// tanhf is a branchy polynomial (~30 VALU ops); the GELU epilogue of the 2048 x 2048
// fc1 GEMM evaluates it 4M times per step.  Saturates exactly (exp -> inf: 1; -> 0:
// -1); max error ~2e-7 absolute, far below the bf16 rounding of the result.
__device__ __forceinline__ float fast_tanh(float u) {
  return 1.0f - 2.0f / (__expf(2.0f * u) + 1.0f);
}

__device__ __forceinline__ float act_fwd(int act, float z) {
  switch (act) {
    case ACT_SILU: return z / (1.0f + __expf(-z));
    case ACT_GELU: {
      const float k = 0.7978845608028654f;  // sqrt(2/pi), tanh approximation (flax nn.gelu default)
      const float t = fast_tanh(k * (z + 0.044715f * z * z * z));
      return 0.5f * z * (1.0f + t);
    }
    case ACT_RELU: return z > 0.f ? z : 0.f;
    default: return z;
  }
}
__device__ __forceinline__ float act_grad(int act, float z) {
  switch (act) {
    case ACT_SILU: {
      const float s = 1.0f / (1.0f + __expf(-z));
      return s * (1.0f + z * (1.0f - s));
    }
    case ACT_GELU: {
      const float k = 0.7978845608028654f;
      const float u = k * (z + 0.044715f * z * z * z);
      const float t = fast_tanh(u);
      const float du = k * (1.0f + 3.0f * 0.044715f * z * z);
      return 0.5f * (1.0f + t) + 0.5f * z * (1.0f - t * t) * du;
    }
    case ACT_RELU: return z > 0.f ? 1.f : 0.f;
    default: return 1.f;
  }
}

// ---------------------------------------------------------------- MFMA wrappers
// D = A(16x32) * B(32x16) + C, bf16 in, f32 accumulate.
// lane l holds A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15]; D[(l>>4)*4+i][l&15].
__device__ __forceinline__ f32x4 mfma16x16x32(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// D = A(32x16) * B(16x32) + C: lane l holds A[l&31][8(l>>5)+j], B[8(l>>5)+j][l&31];
// D register e of lane l is row (e&3) + 8(e>>2) + 4(l>>5), column l&31.  Half the
// fragment bytes per FLOP of the 16x16x32 form (one 16-byte A and B read per 32K FLOP).
__device__ __forceinline__ f32x16 mfma32x32x16(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------- XCD-aware 2-D block map
// Workgroups are dealt round-robin over the 8 XCDs (linear id L -> XCD L % 8), so in
// a grid whose x index walks 16-column output blocks, blocks x and x+1 write the two
// 64-byte halves of every 128-byte line from two different XCD L2s: each L2 writes
// back (and first fetches) a partial line.  This bijection gives every XCD a
// contiguous run of tiles in x-fastest order, so neighbouring column blocks share an
// L2 and the lines leave it whole.  Identity when the grid is not a multiple of 8.
__device__ __forceinline__ void xcd_contiguous_tile(int& bx, int& by) {
  const int gx = gridDim.x, G = gx * gridDim.y;
  const int L = blockIdx.x + gx * blockIdx.y;
  if (G % 8) { bx = blockIdx.x; by = blockIdx.y; return; }
  const int t = (L % 8) * (G / 8) + L / 8;
  bx = t % gx; by = t / gx;
}

// Run-ahead tile map, from the XCD the workgroup actually runs on (HW_REG_XCC_ID):
// XCD x takes tiles [x G/8, (x+1) G/8) in chunk-fastest order, i.e. whole column
// blocks (all gridDim.y input chunks of 16 hidden units: their Z1 partials meet in
// the XCD's L2) and 4 neighbouring ones (whole 128-byte lines of W1 rows); its
// workgroups are told apart by L / 8.  Workgroups are dealt round-robin over the XCDs
// (linear id L -> XCD (L + o) % 8, the offset o carried over from earlier dispatches),
// so each XCD gets G/8 workgroups with distinct L / 8 and this is a bijection.  The
// body checks it: every tile has a per-launch counter (ztick tail) that must read
// the launch number, otherwise the error word is raised and the host refuses the
// results (FusedMLP2 / FusedMLPDeep .finalize).
__device__ __forceinline__ void xcd_column_tile(int& bx, int& by) {
  const int L = blockIdx.x + gridDim.x * blockIdx.y, G = gridDim.x * gridDim.y;
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
  const int t = (int)(xcc & 7u) * (G / 8) + L / 8;
  bx = t / gridDim.y;
  by = t % gridDim.y;
}

// A kernel-argument pointer pinned in SGPRs.  Selecting between struct members with a
// lane-dependent condition (`aux ? a.pW2 : a.pW1`) lets the compiler turn the select
// into a per-lane load of the member's ADDRESS from the kernarg segment: a vector load
// whose result the next loads wait for, and an in-order vmcnt wait also drains every
// load issued before it (one extra global round trip).  readfirstlane makes the
// pointer a uniform value first, so the select is a v_cndmask on registers.
template <class T>
__device__ __forceinline__ T* sgpr_ptr(T* p) {
  const unsigned long long v = reinterpret_cast<unsigned long long>(p);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return reinterpret_cast<T*>(((unsigned long long)hi << 32) | lo);
}
// a load through such a pointer as a global (not flat) access
__device__ __forceinline__ float ld_global(const float* p) {
  return *(const __attribute__((address_space(1))) float*)p;
}

// ---------------------------------------------------------------- system-scope (cross-GPU) payload
// IPC-mapped buffers (comm/csrc: xGMI collectives, pipeline inboxes) are written by one
// GPU and read by another over xGMI.  Their coherence is made explicit on EVERY payload
// instruction instead of being inherited from the memory type the importing GPU's
// mapping happens to get (a peer-VRAM mapping of an ordinary allocation is cached
// non-coherently in the reader's L2, so a re-read of the same address in a later
// call could hit a stale line): accesses are buffer instructions with the
// cache-policy bits sc0 sc1 (aux = 1 | 16), the system-scope form that the LLVM
// AMDGPU memory model for GFX942/GFX950 emits for system-scope relaxed atomics --
//   load  atomic monotonic, system  ->  buffer/global_load  ... sc0 sc1
//   store atomic monotonic, system  ->  buffer/global_store ... sc0 sc1
// -- i.e. a load is served coherently at system scope (no stale L1/L2 copy) and a
// store is written through past this GPU's caches.  Ordering: each storing wave
// drains its stores (s_waitcnt vmcnt(0)) and the workgroup barriers before ONE lane
// raises the peer's flag with a relaxed system-scope atomic store; the reader polls
// that flag with relaxed system-scope atomic loads, barriers, then issues its
// payload loads (all sc0 sc1).  Out-of-range offsets are dropped by the buffer
// bounds check (num_records), never written.
constexpr int CPOL_SYS = 1 | 16;  // sc0 | sc1
typedef __attribute__((ext_vector_type(4))) unsigned sys_u32x4;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t sys_rsrc(const void* base, unsigned long long bytes) {
  const int n = bytes >= 0x7fffffffull ? 0x7fffffff : (int)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, n, 0x00020000);
}
// The same for a base the caller knows to be wave-uniform: readfirstlane pins the whole
// resource in SGPRs.  A base that merely IS uniform can still reach the resource as a
// "divergent" value (a phi after a lane-dependent branch), and a buffer access through
// a VGPR resource compiles into a readfirstlane waterfall loop per instruction.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sys_rsrc_u(const void* base, unsigned long long bytes) {
  const int n = bytes >= 0x7fffffffull ? 0x7fffffff : (int)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(sgpr_ptr(const_cast<void*>(base)), (short)0,
                                           __builtin_amdgcn_readfirstlane(n), 0x00020000);
}
__device__ __forceinline__ float4 sys_load4(__amdgpu_buffer_rsrc_t r, long float_off) {
  const sys_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(float_off * 4), 0, CPOL_SYS);
  return __builtin_bit_cast(float4, v);
}
__device__ __forceinline__ void sys_store4(__amdgpu_buffer_rsrc_t r, long float_off, float4 x) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(sys_u32x4, x), r, (int)(float_off * 4), 0, CPOL_SYS);
}
__device__ __forceinline__ float sys_load1(__amdgpu_buffer_rsrc_t r, long float_off) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)(float_off * 4), 0, CPOL_SYS));
}
__device__ __forceinline__ void sys_store1(__amdgpu_buffer_rsrc_t r, long float_off, float x) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, x), r, (int)(float_off * 4), 0, CPOL_SYS);
}

// ---------------------------------------------------------------- tile exchange (N > 1 run-ahead step)
// The data-parallel step of the fused 2-layer engine at N > 1 as ONE launch per step
// (mlp_fused.hip mlp2_bwd AHEAD with Mlp2Args::tx): every workgroup all-reduces its own
// gradient tile with the same tile of the other ranks' launches -- a two-shot exchange
// per tile (tile T is summed by rank T % W, in rank order, and the sum pushed back to
// every rank) -- then applies AdamW and runs the next step's forward exactly as on one
// GPU.  IPC buffers (comm/csrc/tile_exchange.hip): per rank a partial inbox
// [tile][src][pay] floats, a reduced inbox [tile][pay] floats and an uncached signal
// page: flag[tile * TX_MAX_RANKS + src] (partial of src arrived), then
// flag[tiles * TX_MAX_RANKS + tile] (reduced tile arrived); epochs = optimizer step + 1.
constexpr int TX_MAX_RANKS = 8;
struct TxArgs {
  float* part[TX_MAX_RANKS];      // rank q's partial inbox (IPC-mapped)
  float* red[TX_MAX_RANKS];       // rank q's reduced inbox
  unsigned* flag[TX_MAX_RANKS];   // rank q's signal page
  int rank, world, tiles, pay;    // pay: floats per tile payload
  long long timeout;              // s_memrealtime ticks (100 MHz) per wait
  unsigned* err;                  // this rank's error word (bit 2: a wait timed out)
};

// Two-shot all-reduce of one workgroup's gradient values with the same tile T of the
// other ranks' launches (common.h TxArgs): tile T belongs to rank T % W.  A non-owner
// pushes its values into the owner's partial inbox (system-scope write-through stores,
// drained, then ONE lane raises the owner's flag [T][rank]) and waits for the reduced
// tile; the owner waits for the W - 1 flags, sums in rank order (own values at its rank
// -- so every rank gets bit-identical sums, as comm/csrc/xgmi.hip), pushes the sum into
// every peer's reduced inbox and raises their flags [T].  Each thread moves only its own
// values: n4 float4 at payload offsets p4[] and one scalar at ps (ps < 0: none).  Every
// wait is bounded (s_memrealtime); a timeout sets bit 2 of the error word and the tile
// goes on with what it has (the host raises on the word).
// Flags as GLOBAL (address space 1) accesses: through a generic pointer they compile to
// flat instructions, which count in lgkmcnt as well as vmcnt -- every later LDS wait of
// the wave would then also wait for the flag store's acknowledgement (over xGMI).
typedef __attribute__((address_space(1))) unsigned tx_gu32;
__device__ __forceinline__ unsigned tx_flag_load(const unsigned* f) {
  return __hip_atomic_load((const tx_gu32*)f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void tx_flag_store(unsigned* f, unsigned v) {
  __hip_atomic_store((tx_gu32*)f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ bool tx_wait(const unsigned* f, unsigned epoch, long long timeout, unsigned* err) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while ((int)(tx_flag_load(f) - epoch) < 0) {
    if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > timeout) {
      __hip_atomic_fetch_or((tx_gu32*)err, 4u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

__device__ __forceinline__ void tx_tile(const TxArgs* X, int T, unsigned epoch, int n4, float4 (&v4)[2],
                                        const int (&p4)[2], float& vs, int ps, unsigned* err) {
  // TxArgs lives in device memory the kernel also writes, so its fields come back in VGPRs;
  // readfirstlane makes them (and the peer pointers, sgpr_ptr) scalar -- a buffer resource
  // built from a VGPR value is a readfirstlane waterfall loop around every access
  const int R = __builtin_amdgcn_readfirstlane(X->rank), W = __builtin_amdgcn_readfirstlane(X->world);
  T = __builtin_amdgcn_readfirstlane(T);
  const int own = T % W, tid = threadIdx.x;
  const long pay = __builtin_amdgcn_readfirstlane(X->pay), tiles = __builtin_amdgcn_readfirstlane(X->tiles);
  const unsigned long long tb = (unsigned long long)pay * 4ull;
  if (R != own) {
    const __amdgpu_buffer_rsrc_t dst = sys_rsrc_u(sgpr_ptr(X->part[own]) + ((long)T * TX_MAX_RANKS + R) * pay, tb);
#pragma unroll
    for (int k = 0; k < 2; ++k)
      if (k < n4) sys_store4(dst, p4[k], v4[k]);
    if (ps >= 0) sys_store1(dst, ps, vs);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains its pushes
    __syncthreads();
    if (tid == 0) {
      tx_flag_store(sgpr_ptr(X->flag[own]) + (long)T * TX_MAX_RANKS + R, epoch);
      tx_wait(X->flag[R] + tiles * TX_MAX_RANKS + T, epoch, X->timeout, err);
    }
    __syncthreads();
    const __amdgpu_buffer_rsrc_t src = sys_rsrc_u(sgpr_ptr(X->red[R]) + (long)T * pay, tb);
#pragma unroll
    for (int k = 0; k < 2; ++k)
      if (k < n4) v4[k] = sys_load4(src, p4[k]);
    if (ps >= 0) vs = sys_load1(src, ps);
    return;
  }
  if (tid < W && tid != R) tx_wait(X->flag[R] + (long)T * TX_MAX_RANKS + tid, epoch, X->timeout, err);
  __syncthreads();
  const float* inbox = sgpr_ptr(X->part[R]) + (long)T * TX_MAX_RANKS * pay;
  // the rank-ordered sum, peers' partials loaded 4 ranks at a time (all 4 in flight)
#pragma unroll
  for (int k = 0; k < 3; ++k) {   // k = 0, 1: the float4 slots; k = 2: the scalar
    if (k < 2 ? k >= n4 : ps < 0) continue;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int g = 0; g < TX_MAX_RANKS; g += 4) {
      if (g >= W) break;
      float4 in[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int q = g + u;
        if (q < W && q != R) {
          const __amdgpu_buffer_rsrc_t src = sys_rsrc_u(inbox + (long)q * pay, tb);
          in[u] = k < 2 ? sys_load4(src, p4[k]) : make_float4(sys_load1(src, ps), 0.f, 0.f, 0.f);
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int q = g + u;
        if (q >= W) break;
        const float4 x = q == R ? (k < 2 ? v4[k] : make_float4(vs, 0.f, 0.f, 0.f)) : in[u];
        if (q == 0) acc = x;
        else { acc.x += x.x; acc.y += x.y; acc.z += x.z; acc.w += x.w; }
      }
    }
    if (k < 2) v4[k] = acc;
    else vs = acc.x;
  }
#pragma unroll
  for (int q = 0; q < TX_MAX_RANKS; ++q) {
    if (q >= W || q == R) continue;
    const __amdgpu_buffer_rsrc_t dst = sys_rsrc_u(sgpr_ptr(X->red[q]) + (long)T * pay, tb);
#pragma unroll
    for (int k = 0; k < 2; ++k)
      if (k < n4) sys_store4(dst, p4[k], v4[k]);
    if (ps >= 0) sys_store1(dst, ps, vs);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid < W && tid != R)
    tx_flag_store(X->flag[tid] + tiles * TX_MAX_RANKS + T, epoch);
}


}  // namespace jdt

#define HIP_LAUNCH_CHECK() (int)hipGetLastError()
