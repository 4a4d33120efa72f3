// One GPipe stage's whole training step in ONE persistent launch per rank
// (BASELINE config #4: the 8-stage MLP 784 -> 512 x 8 -> 10, one dense layer per
// stage, the 10-class head on the last stage).
//
// The per-tick path (parallel/pipeline.py _compute_fused) issues, per microbatch and
// direction, a receive kernel, the layer's md_fwd / md_bwd launch, a dX GEMM and a
// send kernel: 3-4 dependent launches of ~4 us each for a 64 x 512 x 512 layer, so a
// tick costs ~13 us and an 8-stage pipeline cannot beat one GPU.  Here the whole
// fill / drain schedule of the step runs inside one launch of 32 workgroups per rank.
// Workgroup b = 2 cb + h owns output columns [32 cb, 32 cb + 32) of the stage's layer
// for rows [h mb/2, (h+1) mb/2) of every microbatch: a hop's input (the previous stage's
// activation, the next stage's dZ) is read once per column block per row half, so each
// workgroup loads half the bytes of a column-only split -- the per-workgroup read rate
// of freshly handed-off data is what bounds a tick (stamps: profiles/r5_pp_intile_stamps.txt).
//
//   step start:      W[:, own] (fp32 master) -> bf16 LDS image; a stage > 0 also writes
//                    its image into its predecessor's weight box (second inbox, by step
//                    parity); stage 0 writes the step's data transposed per microbatch
//                    (X^T, the dW operand; its forward reads the fp32 rows directly)
//   forward tick i:  wait for the flags of the 16 producers of this row half (per wave:
//                    only the 2 whose columns are its k range), Z = X W[:, own] + b on
//                    MFMA (K split over the 8 waves), SiLU, dropout (the md kernels' Philox
//                    streams), backward factor G kept in LDS; H and H^T of the tile go
//                    straight into the NEXT stage's inbox (system-scope stores over xGMI)
//                    and one flag per workgroup is raised -- or, last stage, the head's
//                    partial logits (fp32 atomics, one arrival counter per row half)
//   backward tick i: dH[half, own] = dZ_next W_next[own, :]^T from the successor's dZ
//                    (inbox) and weight image (weight box) on MFMA -- or, last stage, CE
//                    of the complete logits through the head; dZ = dH * G goes straight
//                    to the predecessor's inbox (not stage 0); then dW[:, own] += X^T dZ
//                    over this row half (registers; X^T prefetched ahead of the wait), db
//   end of step:     each row half stores its partial weight gradients; a second, wide
//                    launch (pp_adam_kernel, ~all CUs) sums the two halves and applies
//                    AdamW (gradient scale 1 / n_mb), bf16 shadows, metrics fold, step
//                    advance.  32 workgroups updating a whole layer's p / m / v moved
//                    ~150 KB per CU and took 10-15 us (stamps); spread over the chip it is
//                    a few us plus one launch boundary.
//
// Every wait is on another workgroup that is resident (32 workgroups, all co-resident,
// host-checked) or on a neighbour stage's launch, and bounded (s_memrealtime) into the
// inbox error word.  Flags are epoch-valued (the device optimizer step + 1, read at
// the start), exactly as comm/csrc/p2p.hip's send / receive kernels, so replays need
// no host bookkeeping; slot reuse is race-free by GPipe's own dependencies (the
// producer overwrites slot i of step t+1 only after every gradient of step t arrived).
// Reference semantics: the intended GPipe of /root/reference/pipeline_parallel.py:37-38
// (SURVEY section 3.5); gradients equal the un-split model's (tests/test_grad_scale_gpu.py
// test_pipeline_stage_kernel_adam_scale, tests/test_xgmi_gpu.py).
#include "common.h"

namespace jdt {

constexpr int PS_NT = 512;         // 8 waves (outstanding loads per workgroup)
constexpr int PS_NW = PS_NT / 64;
constexpr int PS_NB = 32;          // workgroups: 16 column blocks x 2 row halves
constexpr int PS_CB = 32;          // columns per workgroup
constexpr int PS_N = 512;          // layer width
constexpr int PS_MAXMB = 64;       // rows per microbatch (32 or 64: 16-row MFMA tiles per half)
constexpr int PS_MAXH = PS_MAXMB / 2;
constexpr int PS_MAXROWS = 128;    // rows per step (n_mb * mb)
constexpr int PS_MAXNMB = 8;
constexpr int PS_C = 10;
constexpr int PS_FLAG_BLOCKS = 32; // comm/csrc/p2p.hip P2P_MAX_BLOCKS (flags per slot)
constexpr int PS_UPWMAX = (784 / 16 + PS_NW - 1) / PS_NW;   // dW k tiles per wave (stage 0: 7)
// partial-gradient slab of one row half (floats, PsArgs::gstride apart): dW [K][512], db
// [512], dW_h [512][C], db_h [C], loss / correct sums (column block 0)
__host__ __device__ constexpr long ps_g_b(int K) { return (long)K * 512; }
__host__ __device__ constexpr long ps_g_wh(int K) { return ps_g_b(K) + 512; }
__host__ __device__ constexpr long ps_g_bh(int K) { return ps_g_wh(K) + 512 * 10; }
__host__ __device__ constexpr long ps_g_met(int K) { return ps_g_bh(K) + 10; }
__host__ __device__ constexpr long ps_g_size(int K) { return ps_g_met(K) + 6; }

struct PsArgs {
  int n_mb, mb;                    // microbatches, rows per microbatch (32 or 64; n_mb * mb = 128)
  int K;                           // layer input width (784: stage 0, else 512)
  int gid;                         // global layer index (dropout stream id)
  int mb_shift;                    // dropout offset of microbatch i: (i << mb_shift) + (gid << 1)
  float keep; unsigned long long seed;
  // layer parameters (fp32 master, Adam moments) and bf16 shadows
  float* p; float* m; float* v; bf16_t* sW;       // W [K][512]
  float* pb; float* mbv; float* vb; bf16_t* sb;   // b [512]
  // head (last stage): W_h [512][C], b_h [C]
  float* ph; float* mh; float* vh; bf16_t* sh;
  float* phb; float* mhb; float* vhb; bf16_t* shb;
  const float* X;                  // stage 0: data [n_mb * mb][784] fp32
  const int* labels;               // last stage: [n_mb * mb]
  // inboxes (comm/csrc/p2p.hip layout): slot i < n_mb: activation of microbatch i (H
  // [mb][512] bf16, then H^T [512][mb]); slot n_mb + i: the successor's dZ [mb][512]
  char* in_mine; unsigned* flag_mine;
  char* in_prev; unsigned* flag_prev;   // rank of stage s-1 (null at stage 0)
  char* in_next; unsigned* flag_next;   // rank of stage s+1 (null at the last stage)
  long slot_bytes;
  int* err;                        // this rank's inbox error word (a wait timed out)
  long long timeout;               // s_memrealtime ticks per wait
  // scratch (zero-initialised once by the host)
  bf16_t* XT;                      // stage 0: X^T [n_mb][784][mb] bf16 (the dW operand)
  // weight boxes (a second p2p inbox of two PS_WBYTES slots, by step parity): a stage > 0
  // writes the bf16 image of its W [512][512] into its predecessor's box at the start of
  // the step; the predecessor's backward forms dH = dZ_next W_next^T itself, so a backward
  // hop carries dZ and no stage waits on an intra-stage gather before sending
  char* w_mine; unsigned* wflag_mine;
  char* w_prev; unsigned* wflag_prev;
  float* logits;                   // last stage: [2][n_mb][mb][C] fp32, by step parity
  unsigned* ctr;                   // arrival counters, one 128-byte line each
  float* gpart; long gstride;      // [2 row halves][gstride] partial gradients (ps_g_*)
  int* step; unsigned* ticket;     // device optimizer step, end-of-step ticket
  float lr, b1, b2, eps, wd, gscale;
  float* mslot; float* running;    // last stage: metric slots (loss, n, correct, n), running sums
  unsigned long long* stamps;      // diagnostic: [32][32] s_memrealtime (null = off)
};

#define PS_STAMP(k)                                                                           \
  do {                                                                                        \
    if (a.stamps && threadIdx.x == 0) a.stamps[(long)b * 32 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

constexpr int CPOL_SC1 = 16;       // agent-coherent (write-through / past L1) buffer access
constexpr long PS_WBYTES = (long)PS_N * PS_N * 2;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t ps_rsrc(const void* base, long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(sgpr_ptr(const_cast<void*>(base)), (short)0,
                                           __builtin_amdgcn_readfirstlane((int)bytes), 0x00020000);
}
template <int CPOL>
__device__ __forceinline__ u32x4 ps_load16(__amdgpu_buffer_rsrc_t r, long byte_off) {
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte_off, 0, CPOL));
}
template <int CPOL>
__device__ __forceinline__ void ps_store16(__amdgpu_buffer_rsrc_t r, long byte_off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(sys_u32x4, v), r, (int)byte_off, 0, CPOL);
}
__device__ __forceinline__ void ps_store8(__amdgpu_buffer_rsrc_t r, long byte_off, unsigned lo, unsigned hi, int cpol_sys) {
  const __attribute__((ext_vector_type(2))) unsigned v = {lo, hi};
  if (cpol_sys) __builtin_amdgcn_raw_buffer_store_b64(v, r, (int)byte_off, 0, CPOL_SYS);
  else __builtin_amdgcn_raw_buffer_store_b64(v, r, (int)byte_off, 0, CPOL_SC1);
}

// this rank's error word: once a wait timed out, every later wait of the step gives up
// at once (the results are refused by the host anyway), so a dead peer costs one timeout
__device__ __forceinline__ bool ps_failed(const int* err) {
  return __hip_atomic_load((const __attribute__((address_space(1))) int*)err, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM) != 0;
}

__device__ __forceinline__ void ps_poll(const unsigned* f, unsigned epoch, long long timeout, int* err) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while ((int)(tx_flag_load(f) - epoch) < 0) {
    if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > timeout) {
      __hip_atomic_store((__attribute__((address_space(1))) int*)err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// Wait until all PS_FLAG_BLOCKS producer flags of `slot` reached `epoch` (wave 0, one
// lane per flag), then the workgroup barrier.  Bounded: a timeout raises *err.
__device__ __forceinline__ void ps_wait_slot(const unsigned* flags, int slot, unsigned epoch, long long timeout,
                                             int* err) {
  if (threadIdx.x < PS_FLAG_BLOCKS && !ps_failed(err))
    ps_poll(flags + (long)slot * PS_FLAG_BLOCKS + threadIdx.x, epoch, timeout, err);
  __syncthreads();
}

// Wave w's share of a 512-deep product (k in [64w, 64w + 64)) comes from the producers
// of column blocks 2w and 2w + 1 in row half h (workgroups 4w + h, 4w + 2 + h): two lanes
// poll just those flags, no workgroup barrier (the data loads that follow are issued
// after the loop exits: in-order issue per wave).
__device__ __forceinline__ void ps_wait_wave(const unsigned* flags, int slot, int h, unsigned epoch,
                                             long long timeout, int* err) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane < 2 && !ps_failed(err))
    ps_poll(flags + (long)slot * PS_FLAG_BLOCKS + 4 * w + 2 * lane + h, epoch, timeout, err);
  asm volatile("" ::: "memory");
}

// This workgroup's stores are drained, then ONE lane raises its flag of `slot` on the peer.
__device__ __forceinline__ void ps_raise(unsigned* peer_flags, int slot, unsigned epoch, int b) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) tx_flag_store(peer_flags + (long)slot * PS_FLAG_BLOCKS + b, epoch);
}

// `cnt` workgroups arrive at counter line `c` (stores drained, one agent-scope add each);
// the target -- the next multiple of cnt above this workgroup's own ticket, so the counter
// never needs a reset -- is returned (lane 0 of wave 0) for a later ps_wait: work placed
// between the two overlaps the other workgroups' arrival.
__device__ __forceinline__ unsigned ps_arrive(unsigned* ctr, int c, unsigned cnt) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  unsigned target = 0;
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(ctr + 32 * c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    target = (old / cnt + 1u) * cnt;
  }
  return target;
}
__device__ __forceinline__ void ps_wait(unsigned* ctr, int c, unsigned target, long long timeout, int* err) {
  if (threadIdx.x == 0) {
    const __amdgpu_buffer_rsrc_t cr = __builtin_amdgcn_make_buffer_rsrc(ctr + 32 * c, (short)0, 4, 0x00020000);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    // (the error word -- a system-scope load -- only every 64th poll: it would set the poll
    // period)
    for (unsigned spins = 0; (int)((unsigned)__builtin_amdgcn_raw_buffer_load_b32(cr, 0, 0, CPOL_SC1) - target) < 0;
         ++spins) {
      if ((spins & 63) == 63 && ps_failed(err)) break;
      if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > timeout) {
        __hip_atomic_store((__attribute__((address_space(1))) int*)err, 2, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      asm volatile("" ::: "memory");
    }
  }
  __syncthreads();
}

// counter lines: stage 0's X^T pre-pass done; logits of microbatch i, row half h complete
// (last stage)
__device__ __forceinline__ int ps_ctr_xt() { return 0; }
__device__ __forceinline__ int ps_ctr_lg(int i, int h) { return 8 + 2 * i + h; }

// LDS of one stage role, carved from one buffer (the one-GPU chain kernel runs every role
// in one launch: static __shared__ arrays of three inlined roles would be summed, a
// carved buffer is their maximum)
__host__ __device__ constexpr int ps_al16(int x) { return (x + 15) & ~15; }
template <bool FIRST, bool LAST>
struct PsLds {
  static constexpr int K = FIRST ? 784 : PS_N;
  static constexpr int LDWC = (K + 31) / 32 * 32 + 8, LDWR = PS_N + 8, LDT = 32 + 8;
  static constexpr int wc = 0;
  static constexpr int wr = ps_al16(wc + PS_CB * LDWC * 2);
  static constexpr int part = ps_al16(wr + (LAST ? 8 : PS_CB * LDWR) * 2);
  static constexpr int gl = ps_al16(part + PS_NW * PS_MAXH * (PS_CB + 1) * 4);
  static constexpr int ht = ps_al16(gl + (PS_MAXROWS / 2) * PS_CB * 4);
  static constexpr int hown = ps_al16(ht + PS_MAXH * (PS_CB + 8) * 2);
  static constexpr int dzT = ps_al16(hown + (LAST ? PS_MAXROWS / 2 : 1) * PS_CB * 2);
  static constexpr int dlog = ps_al16(dzT + PS_CB * LDT * 2);
  static constexpr int whs = ps_al16(dlog + (LAST ? PS_MAXH : 1) * (PS_C + 1) * 4);
  static constexpr int bsh = ps_al16(whs + PS_CB * PS_C * 4);
  static constexpr int red = ps_al16(bsh + PS_CB * 4);
  static constexpr int tgt = ps_al16(red + 2 * PS_NW * 4);
  static constexpr int size = ps_al16(tgt + PS_MAXNMB * 4);
};
constexpr int ps_max3(int x, int y, int z) { return x > y ? (x > z ? x : z) : (y > z ? y : z); }
constexpr int PS_LDS_MAX = ps_max3(PsLds<true, false>::size, PsLds<false, false>::size, PsLds<false, true>::size);

// One stage's step, workgroup b of the stage's PS_NB (the per-rank launch: blockIdx.x;
// the one-GPU chain: blockIdx.x % PS_NB), over the LDS buffer `lds`.
template <bool FIRST, bool LAST>
__device__ __forceinline__ void ps_body(const PsArgs& a, const int b, char* __restrict__ lds) {
  constexpr int K = FIRST ? 784 : PS_N;
  constexpr int KS = (K + 31) / 32;             // 32-deep k-steps of the forward
  constexpr int KP = KS * 32;
  constexpr int LDWC = KP + 8;                  // padded LDS rows (bank spread)
  constexpr int LDWR = PS_N + 8;
  constexpr int NTK = K / 16;                   // 16-wide k tiles of dW^T (49 or 32)
  constexpr int NTK_H = (NTK + 1) / 2;          // row half 0 updates k tiles [0, NTK_H)
  constexpr int UPW = (NTK + PS_NW - 1) / PS_NW; // dW^T k tiles per wave
  constexpr int TPW = (KS + PS_NW - 1) / PS_NW;  // forward k-steps per wave
  constexpr int KSW = (PS_N / 32) / PS_NW;      // k-steps per wave of a 512-deep product
  constexpr int MTH = PS_MAXH / 16;             // 16-row tiles of a row half (max)
  constexpr int LDT = 32 + 8;                   // dzT rows: 32 (the dW k-step; half rows + zeros)
  static_assert(K % 16 == 0 && UPW <= PS_UPWMAX, "dW tiles");
  static_assert(KSW * 32 == 64 && PS_NW * 64 == PS_N, "a wave's k range = two producers' column blocks");
  using LL = PsLds<FIRST, LAST>;
  static_assert(LL::LDWC == LDWC && LL::LDT == LDT, "LDS layout");
  bf16_t* const wc = reinterpret_cast<bf16_t*>(lds + LL::wc);                      // W[:, own]^T
  bf16_t* const wr = reinterpret_cast<bf16_t*>(lds + LL::wr);                      // W_next[own rows, :]
  float(*const part)[PS_MAXH][PS_CB + 1] = reinterpret_cast<float(*)[PS_MAXH][PS_CB + 1]>(lds + LL::part);
  float(*const gl)[PS_CB] = reinterpret_cast<float(*)[PS_CB]>(lds + LL::gl);      // G of own rows / cols
  bf16_t(*const ht)[PS_CB + 8] = reinterpret_cast<bf16_t(*)[PS_CB + 8]>(lds + LL::ht);   // this tick's H tile
  bf16_t(*const hown)[PS_CB] = reinterpret_cast<bf16_t(*)[PS_CB]>(lds + LL::hown);       // head input
  bf16_t* const dzT = reinterpret_cast<bf16_t*>(lds + LL::dzT);                    // dZ[half, own]^T
  float(*const dlog)[PS_C + 1] = reinterpret_cast<float(*)[PS_C + 1]>(lds + LL::dlog);
  float(*const whs)[PS_C] = reinterpret_cast<float(*)[PS_C]>(lds + LL::whs);
  float* const bsh = reinterpret_cast<float*>(lds + LL::bsh);
  float(*const red)[PS_NW] = reinterpret_cast<float(*)[PS_NW]>(lds + LL::red);
  unsigned* const tgt = reinterpret_cast<unsigned*>(lds + LL::tgt);                // counter targets (lane 0)

  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cb = b >> 1, h = b & 1, j0 = PS_CB * cb;
  const int mb = a.mb, n_mb = a.n_mb, mh = mb >> 1, MT = mh / 16;
  const int step = a.step[0], par = step & 1;
  const unsigned epoch = (unsigned)step + 1u;
  const unsigned long long dbase = (unsigned long long)(unsigned)step << 32;
  const float rkeep = 1.f / a.keep;
  PS_STAMP(0);

  // ---- 0. this step's weights into LDS (bf16 rounding of the fp32 masters = the
  // shadows): every load first, then the images; stage 0's data rows for the X^T
  // pre-pass load with them
  static_assert(!FIRST || K / 4 <= PS_NT, "one float4 column per thread");
  float4 xpre[FIRST ? 4 : 1];
  // the forward's k-steps of this wave: [w KS / 8, (w+1) KS / 8) of every 16-row tile
  const int ks0 = (w * KS) / PS_NW, ks1 = ((w + 1) * KS) / PS_NW;
  // stage 0: the fp32 data rows of microbatch i's row half for this wave's k-steps
  // (software-pipelined: microbatch i + 1's loads fly during tick i).  k past 784 (the
  // 25th k-step's upper half) reads the next row or, past the buffer, zero (bounds
  // check): finite values times wc's zero padding
  float4 xf[FIRST ? MTH : 1][FIRST ? TPW : 1][2];
  auto load_x = [&](int i) {
    if constexpr (FIRST) {
      const int r0 = i * mb + h * mh;
      const __amdgpu_buffer_rsrc_t xr = ps_rsrc(a.X + (long)r0 * K, (long)(PS_MAXROWS - r0) * K * 4);
#pragma unroll
      for (int t = 0; t < TPW; ++t)
#pragma unroll
        for (int mt = 0; mt < MTH; ++mt) {
          if (mt >= MT) continue;
          const int ks = min(ks0 + t, ks1 - 1), row = mt * 16 + (lane & 15);
          const long off = ((long)row * K + ks * 32 + 8 * (lane >> 4)) * 4;
          xf[mt][t][0] = __builtin_bit_cast(float4, ps_load16<0>(xr, off));
          xf[mt][t][1] = __builtin_bit_cast(float4, ps_load16<0>(xr, off + 16));
        }
    }
  };
  load_x(0);
  {
    constexpr int WC4 = (K * (PS_CB / 4) + PS_NT - 1) / PS_NT;   // float4 of W[:, own] per thread
    float4 wv[WC4];
#pragma unroll
    for (int t = 0; t < WC4; ++t) {
      const int idx = min(tid + t * PS_NT, K * (PS_CB / 4) - 1);
      wv[t] = *reinterpret_cast<const float4*>(a.p + (long)(idx >> 3) * PS_N + j0 + 4 * (idx & 7));
    }
    if constexpr (FIRST) {
      if (tid < K / 4)
#pragma unroll
        for (int e = 0; e < 4; ++e) xpre[e] = *reinterpret_cast<const float4*>(a.X + (long)(4 * b + e) * K + 4 * tid);
    }
    const float bv = a.pb[j0 + (tid & 31)];
    float hv = 0.f;
    if constexpr (LAST) {
      const int t = min(tid, PS_CB * PS_C - 1);
      hv = a.ph[(long)(j0 + t / PS_C) * PS_C + t % PS_C];
    }
#pragma unroll
    for (int t = 0; t < WC4; ++t) {
      const int idx = tid + t * PS_NT;
      if (idx < K * (PS_CB / 4)) {
        const int k = idx >> 3, q = idx & 7;
        wc[(4 * q + 0) * LDWC + k] = f2bf(wv[t].x);
        wc[(4 * q + 1) * LDWC + k] = f2bf(wv[t].y);
        wc[(4 * q + 2) * LDWC + k] = f2bf(wv[t].z);
        wc[(4 * q + 3) * LDWC + k] = f2bf(wv[t].w);
      }
    }
    if constexpr (KP > K)
      for (int idx = tid; idx < PS_CB * (KP - K); idx += PS_NT) wc[(idx / (KP - K)) * LDWC + K + idx % (KP - K)] = 0;
    if constexpr (!FIRST) {
      // W[:, own] (bf16) into the predecessor's weight box, slot = step parity (row half h
      // writes rows [h K/2, (h+1) K/2)); its flag goes up after the forward ticks (their
      // sends drain these stores too)
      const __amdgpu_buffer_rsrc_t wo = ps_rsrc(a.w_prev + (long)par * PS_WBYTES, PS_WBYTES);
#pragma unroll
      for (int t = 0; t < WC4; ++t) {
        const int idx = tid + t * PS_NT;
        const int k = idx >> 3, q = idx & 7;
        if (idx < K * (PS_CB / 4) && (k >= K / 2) == (h == 1)) {
          const unsigned lo = (unsigned)f2bf(wv[t].x) | ((unsigned)f2bf(wv[t].y) << 16);
          const unsigned hi = (unsigned)f2bf(wv[t].z) | ((unsigned)f2bf(wv[t].w) << 16);
          ps_store8(wo, ((long)k * PS_N + j0 + 4 * q) * 2, lo, hi, 1);
        }
      }
    }
    if (tid < PS_CB) bsh[tid] = round_bf(bv);
    if constexpr (LAST) {
      if (tid < PS_CB * PS_C) whs[tid / PS_C][tid % PS_C] = round_bf(hv);
      // re-arm the other parity's logit accumulator (the previous step's, fully consumed)
      if (b == 0)
        for (int idx = tid; idx < n_mb * mb * PS_C; idx += PS_NT) a.logits[(long)(par ^ 1) * PS_MAXROWS * PS_C + idx] = 0.f;
    }
  }
  // stage 0: the step's data transposed per microbatch (the dW operand): workgroup b
  // converts rows [4b, 4b + 4) (n_mb * mb == 128, host-checked), write-through; waited
  // for before the first backward tick
  unsigned t_xt = 0;
  if constexpr (FIRST) {
    const int rr = 4 * b, i = rr / mb, rl = rr - i * mb;
    if (tid < K / 4) {
      const __amdgpu_buffer_rsrc_t xtr = ps_rsrc(a.XT + (long)i * K * mb, (long)K * mb * 2);
      const float* xs = &xpre[0].x;
#pragma unroll
      for (int c = 0; c < 4; ++c) {   // feature 4 tid + c of the 4 rows: 8 contiguous bytes of X^T
        const unsigned lo = (unsigned)f2bf(xs[0 * 4 + c]) | ((unsigned)f2bf(xs[1 * 4 + c]) << 16);
        const unsigned hi = (unsigned)f2bf(xs[2 * 4 + c]) | ((unsigned)f2bf(xs[3 * 4 + c]) << 16);
        ps_store8(xtr, ((long)(4 * tid + c) * mb + rl) * 2, lo, hi, 0);
      }
    }
    t_xt = ps_arrive(a.ctr, ps_ctr_xt(), PS_NB);
  } else {
    __syncthreads();
  }
  PS_STAMP(1);

  // ---- 1. forward ticks
  for (int i = 0; i < n_mb; ++i) {
    const int r0 = i * mb + h * mh;   // this workgroup's rows of the step
    // this thread's dropout bits (4 rows x 1 column) do not wait for the inputs
    const int g4 = tid >> 5, c = tid & 31;
    u32x4 db = {0u, 0u, 0u, 0u};
    if (a.keep < 1.f && 4 * g4 < mh) {
      const unsigned long long off = (unsigned long long)((long)i << a.mb_shift) + ((unsigned long long)a.gid << 1);
      db = dropout_bits(a.seed, off + dbase, dropout_group(0, h * mh + 4 * g4, j0 + c, mb, PS_N));
    }
    if constexpr (!FIRST) ps_wait_wave(a.flag_mine, i, h, epoch, a.timeout, a.err);
    if (i == 1) PS_STAMP(19);
    // Z partials: wave w takes its k-steps of both 16-column tiles of every 16-row tile;
    // all of its A fragments are loaded first (stage 0: the fp32 data rows, converted in
    // registers; else the inbox slot written by the previous stage)
    f32x4 acc[MTH][2];
#pragma unroll
    for (int mt = 0; mt < MTH; ++mt) acc[mt][0] = acc[mt][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
    {
      bf16x8 af[MTH][TPW];
      if constexpr (FIRST) {
#pragma unroll
        for (int t = 0; t < TPW; ++t)
#pragma unroll
          for (int mt = 0; mt < MTH; ++mt) {
            if (mt >= MT) continue;
            const float* f = &xf[mt][t][0].x;
#pragma unroll
            for (int q = 0; q < 8; ++q) af[mt][t][q] = (short)f2bf(f[q]);
          }
        if (i + 1 < n_mb) load_x(i + 1);
      } else {
        const __amdgpu_buffer_rsrc_t xin = ps_rsrc(a.in_mine + (long)i * a.slot_bytes, (long)mb * PS_N * 2);
#pragma unroll
        for (int t = 0; t < TPW; ++t)
#pragma unroll
          for (int mt = 0; mt < MTH; ++mt) {
            if (mt >= MT) continue;
            const int ks = min(ks0 + t, ks1 - 1), row = h * mh + mt * 16 + (lane & 15);
            af[mt][t] = __builtin_bit_cast(
                bf16x8, ps_load16<CPOL_SYS>(xin, ((long)row * K + ks * 32 + 8 * (lane >> 4)) * 2));
          }
      }
#pragma unroll
      for (int t = 0; t < TPW; ++t) {
        const int ks = ks0 + t;
        if (ks >= ks1) break;
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
          const bf16x8 bf =
              *reinterpret_cast<const bf16x8*>(&wc[(ct * 16 + (lane & 15)) * LDWC + ks * 32 + 8 * (lane >> 4)]);
#pragma unroll
          for (int mt = 0; mt < MTH; ++mt)
            if (mt < MT) acc[mt][ct] = mfma16x16x32(af[mt][t], bf, acc[mt][ct]);
        }
      }
    }
#pragma unroll
    for (int mt = 0; mt < MTH; ++mt)
      if (mt < MT)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
          for (int e = 0; e < 4; ++e) part[w][mt * 16 + (lane >> 4) * 4 + e][ct * 16 + (lane & 15)] = acc[mt][ct][e];
    __syncthreads();
    if (i == 1) PS_STAMP(20);
    // bias + SiLU + dropout, one 4-row group x 1 column per thread (the md kernels' streams)
    if (4 * g4 < mh) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int rl = 4 * g4 + e;
        float v = bsh[c];
#pragma unroll
        for (int q = 0; q < PS_NW; ++q) v += part[q][rl][c];
        const float z = round_bf(v);
        const float ez = __expf(-z), sg = 1.0f / (1.0f + ez);
        float hv = z * sg, gd = sg * (1.0f + z * (1.0f - sg));
        if (a.keep < 1.f) {
          const bool kp = keep_word(db, e, a.keep);
          hv = kp ? hv * rkeep : 0.f;
          gd = kp ? gd * rkeep : 0.f;
        }
        gl[i * mh + rl][c] = gd;
        const bf16_t hb = f2bf(hv);
        ht[rl][c] = hb;
        if constexpr (LAST) hown[i * mh + rl][c] = hb;
      }
    }
    __syncthreads();
    if (i == 1) PS_STAMP(21);
    if constexpr (LAST) {
      // the head's partial logits of the owned 32 hidden units for this row half (+ b_h
      // from column block 0); the arrival is waited for in the backward
      float* lg = a.logits + (long)par * PS_MAXROWS * PS_C + (long)r0 * PS_C;
      if (tid < mh * PS_C) {
        const int r = tid / PS_C, cc = tid % PS_C;
        float s = cb == 0 ? round_bf(a.phb[cc]) : 0.f;
#pragma unroll
        for (int n = 0; n < PS_CB; ++n) s += bf2f(ht[r][n]) * whs[n][cc];
        // a RETURNING add: waiting for the old value proves the add was performed at the
        // memory side before the arrival below (a no-return add's acknowledgement does not:
        // profiles/r5_pst_headline.txt, the persistent headline kernel's lesson)
        const float old = __hip_atomic_fetch_add((__attribute__((address_space(1))) float*)(lg + tid), s,
                                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("" ::"v"(old));
      }
      const unsigned t_ = ps_arrive(a.ctr, ps_ctr_lg(i, h), PS_NB / 2);
      if (tid == 0) tgt[i] = t_;
    } else {
      // H[half, own] and H^T[own, half] into the next stage's inbox slot i, then this
      // workgroup's flag
      const __amdgpu_buffer_rsrc_t o = ps_rsrc(a.in_next + (long)i * a.slot_bytes, a.slot_bytes);
      if (tid < mh * 4) {
        const int r = tid >> 2, q = tid & 3;
        ps_store16<CPOL_SYS>(o, ((long)(h * mh + r) * PS_N + j0 + 8 * q) * 2, *reinterpret_cast<const u32x4*>(&ht[r][8 * q]));
      }
      const long tbase = (long)mb * PS_N * 2;
      if (tid < PS_CB * (mh / 8)) {
        const int n = tid / (mh / 8), r8 = (tid % (mh / 8)) * 8;
        unsigned q[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) q[e] = (unsigned)ht[r8 + 2 * e][n] | ((unsigned)ht[r8 + 2 * e + 1][n] << 16);
        ps_store16<CPOL_SYS>(o, tbase + ((long)(j0 + n) * mb + h * mh + r8) * 2, (u32x4){q[0], q[1], q[2], q[3]});
      }
      ps_raise(a.flag_next, i, epoch, b);
    }
    if (i < 8) PS_STAMP(2 + i);
  }

  // the weight image written at the start is drained by now (every send waited on it)
  if constexpr (!FIRST) ps_raise(a.wflag_prev, par, epoch, b);
  // the successor's W rows of this workgroup's columns: wr[r][j] = W_next[j0 + r][j]
  if constexpr (!LAST) {
    ps_wait_slot(a.wflag_mine, par, epoch, a.timeout, a.err);
    const __amdgpu_buffer_rsrc_t wi = ps_rsrc(a.w_mine + (long)par * PS_WBYTES, PS_WBYTES);
    constexpr int WN16 = PS_CB * PS_N / 8 / PS_NT;   // 16-byte chunks per thread
    u32x4 q[WN16];
#pragma unroll
    for (int t = 0; t < WN16; ++t) {
      const int idx = tid + t * PS_NT, r = idx >> 6, c8 = (idx & 63) * 8;
      q[t] = ps_load16<CPOL_SYS>(wi, ((long)(j0 + r) * PS_N + c8) * 2);
    }
#pragma unroll
    for (int t = 0; t < WN16; ++t) {
      const int idx = tid + t * PS_NT, r = idx >> 6, c8 = (idx & 63) * 8;
      *reinterpret_cast<u32x4*>(&wr[r * LDWR + c8]) = q[t];
    }
    __syncthreads();
  }
  if constexpr (FIRST) ps_wait(a.ctr, ps_ctr_xt(), t_xt, a.timeout, a.err);   // X^T complete

  // ---- 2. backward ticks, last microbatch first
  f32x4 dwa[UPW][2];
#pragma unroll
  for (int u = 0; u < UPW; ++u) dwa[u][0] = dwa[u][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float dba = 0.f;                   // threads < 32: db[j0 + tid] over this row half
  float dwh = 0.f, dbh = 0.f;        // last stage: threads < 320: dW_h[j0 + t/C][t%C]; cb == 0, t < C: db_h
  float l_loss = 0.f, l_corr = 0.f;
  for (int i = n_mb - 1; i >= 0; --i) {
    const int r0 = i * mb + h * mh;
    // the dW operand (X^T columns of this row half of microbatch i: stage 0's transposed
    // copy, else the inbox slot's H^T part) is already there: its loads fly while this
    // tick waits for dZ_next.  32 columns per k-step: for mh = 16 the upper 16 belong to
    // the other half (or past the slot: zero) and meet dzT's zero rows
    const bf16_t* xtb = FIRST ? a.XT + (long)i * K * mb
                              : reinterpret_cast<const bf16_t*>(a.in_mine + (long)i * a.slot_bytes + (long)mb * PS_N * 2);
    const __amdgpu_buffer_rsrc_t xr = ps_rsrc(xtb, (long)K * mb * 2);
    bf16x8 xb[UPW];
#pragma unroll
    for (int u = 0; u < UPW; ++u) {
      const int t = min(w + PS_NW * u, NTK - 1);
      const long off = ((long)(16 * t + (lane & 15)) * mb + h * mh + 8 * (lane >> 4)) * 2;
      xb[u] = FIRST ? __builtin_bit_cast(bf16x8, ps_load16<CPOL_SC1>(xr, off))
                    : __builtin_bit_cast(bf16x8, ps_load16<CPOL_SYS>(xr, off));
    }
    // dH[half, own] -> dZ = dH * G -> dzT (bf16, as the md kernels round dZ)
    if constexpr (LAST) {
      ps_wait(a.ctr, ps_ctr_lg(i, h), tgt[i], a.timeout, a.err);
      // CE of this row half of microbatch i from the complete logits
      const __amdgpu_buffer_rsrc_t lr =
          ps_rsrc(a.logits + (long)par * PS_MAXROWS * PS_C + (long)r0 * PS_C, (long)mh * PS_C * 4);
      if (tid < mh) {
        float lrow[PS_C];
#pragma unroll
        for (int cc = 0; cc < PS_C; ++cc)
          lrow[cc] = round_bf(__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(lr, (tid * PS_C + cc) * 4, 0,
                                                                                              CPOL_SC1)));
        const int lab = a.labels[r0 + tid];
        float mx = -INFINITY;
        int am = 0;
#pragma unroll
        for (int cc = 0; cc < PS_C; ++cc)
          if (lrow[cc] > mx) { mx = lrow[cc]; am = cc; }
        float s = 0.f;
#pragma unroll
        for (int cc = 0; cc < PS_C; ++cc) s += __expf(lrow[cc] - mx);
        const float lse = mx + __logf(s);
        float ll = 0.f;   // lrow[lab] without a dynamically indexed (scratch) array
#pragma unroll
        for (int cc = 0; cc < PS_C; ++cc) ll = cc == lab ? lrow[cc] : ll;
        l_loss += lse - ll;
        l_corr += (am == lab) ? 1.f : 0.f;
        const float inv = 1.f / (float)mb;
#pragma unroll
        for (int cc = 0; cc < PS_C; ++cc)
          dlog[tid][cc] = round_bf((__expf(lrow[cc] - lse) - (cc == lab ? 1.f : 0.f)) * inv);
      }
      __syncthreads();
      {
        const int g4 = tid >> 5, c = tid & 31;
        if (4 * g4 < mh) {
          unsigned pk[2] = {0u, 0u};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int rl = 4 * g4 + e;
            float dh = 0.f;
#pragma unroll
            for (int k = 0; k < PS_C; ++k) dh += dlog[rl][k] * whs[c][k];
            pk[e >> 1] |= (unsigned)f2bf(dh * gl[i * mh + rl][c]) << (16 * (e & 1));
          }
          *reinterpret_cast<uint2*>(&dzT[c * LDT + 4 * g4]) = make_uint2(pk[0], pk[1]);
        }
      }
      // head gradients of the owned rows of W_h over this row half (b_h: column block 0)
      if (tid < PS_CB * PS_C) {
        const int n = tid / PS_C, cc = tid % PS_C;
        float s = 0.f;
        for (int r = 0; r < mh; ++r) s += bf2f(hown[i * mh + r][n]) * dlog[r][cc];
        dwh += s;
      }
      if (cb == 0 && tid < PS_C) {
        float s = 0.f;
        for (int r = 0; r < mh; ++r) s += dlog[r][tid];
        dbh += s;
      }
    } else {
      // dH[half, own] = dZ_next W_next[own, :]^T: the successor's dZ (inbox slot n_mb + i)
      // is the A operand; wave w takes k-steps [2w, 2w + 2) of the 512-deep product
      ps_wait_wave(a.flag_mine, n_mb + i, h, epoch, a.timeout, a.err);
      const __amdgpu_buffer_rsrc_t gin = ps_rsrc(a.in_mine + (long)(n_mb + i) * a.slot_bytes, (long)mb * PS_N * 2);
      bf16x8 za[MTH][KSW];
#pragma unroll
      for (int t = 0; t < KSW; ++t)
#pragma unroll
        for (int mt = 0; mt < MTH; ++mt) {
          if (mt >= MT) continue;
          za[mt][t] = __builtin_bit_cast(
              bf16x8, ps_load16<CPOL_SYS>(gin, ((long)(h * mh + mt * 16 + (lane & 15)) * PS_N + (KSW * w + t) * 32 +
                                                8 * (lane >> 4)) * 2));
        }
      f32x4 acc[MTH][2];
#pragma unroll
      for (int mt = 0; mt < MTH; ++mt) acc[mt][0] = acc[mt][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < KSW; ++t)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
          const bf16x8 bf = *reinterpret_cast<const bf16x8*>(
              &wr[(ct * 16 + (lane & 15)) * LDWR + (KSW * w + t) * 32 + 8 * (lane >> 4)]);
#pragma unroll
          for (int mt = 0; mt < MTH; ++mt)
            if (mt < MT) acc[mt][ct] = mfma16x16x32(za[mt][t], bf, acc[mt][ct]);
        }
#pragma unroll
      for (int mt = 0; mt < MTH; ++mt)
        if (mt < MT)
#pragma unroll
          for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int e = 0; e < 4; ++e) part[w][mt * 16 + (lane >> 4) * 4 + e][ct * 16 + (lane & 15)] = acc[mt][ct][e];
      __syncthreads();
      // dZ = bf16(bf16(dH) * G), the rounding points of the per-tick path (dX sent as bf16)
      const int g4 = tid >> 5, c = tid & 31;
      if (4 * g4 < mh) {
        unsigned pk[2] = {0u, 0u};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int rl = 4 * g4 + e;
          float v = 0.f;
#pragma unroll
          for (int q = 0; q < PS_NW; ++q) v += part[q][rl][c];
          pk[e >> 1] |= (unsigned)f2bf(round_bf(v) * gl[i * mh + rl][c]) << (16 * (e & 1));
        }
        *reinterpret_cast<uint2*>(&dzT[c * LDT + 4 * g4]) = make_uint2(pk[0], pk[1]);
      }
    }
    if (i == 1) PS_STAMP(22);
    // zero rows [mh, 32) of dzT for the 32-deep dW k-step
    for (int idx = tid; idx < PS_CB * (32 - mh); idx += PS_NT) dzT[(idx / (32 - mh)) * LDT + mh + idx % (32 - mh)] = 0;
    __syncthreads();
    if (tid < PS_CB) {
      float s = 0.f;
      for (int r = 0; r < mh; ++r) s += bf2f(dzT[tid * LDT + r]);
      dba += s;
    }
    // dZ[half, own] to the predecessor (stage 0's input needs no gradient), then dW
    if constexpr (!FIRST) {
      const __amdgpu_buffer_rsrc_t o = ps_rsrc(a.in_prev + (long)(n_mb + i) * a.slot_bytes, (long)mb * PS_N * 2);
      if (tid < mh * 4) {
        const int r = tid >> 2, q8 = (tid & 3) * 8;
        unsigned q[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          q[e] = (unsigned)dzT[(q8 + 2 * e) * LDT + r] | ((unsigned)dzT[(q8 + 2 * e + 1) * LDT + r] << 16);
        ps_store16<CPOL_SYS>(o, ((long)(h * mh + r) * PS_N + j0 + q8) * 2, (u32x4){q[0], q[1], q[2], q[3]});
      }
      ps_raise(a.flag_prev, n_mb + i, epoch, b);
    }
    // dW^T[own cols][k] += dZ^T X over this row half (A = dzT, B = the prefetched X^T
    // columns); wave w takes k tiles w, w + 8, ..., both 16-column tiles
    {
      bf16x8 dza[2];
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
        dza[ct] = *reinterpret_cast<const bf16x8*>(&dzT[(ct * 16 + (lane & 15)) * LDT + 8 * (lane >> 4)]);
#pragma unroll
      for (int u = 0; u < UPW; ++u) {
        if (w + PS_NW * u >= NTK) break;
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) dwa[u][ct] = mfma16x16x32(dza[ct], xb[u], dwa[u][ct]);
      }
    }
    if (i == 1) PS_STAMP(23);
    __syncthreads();
    if (i < 8) PS_STAMP(10 + i);
  }

  // ---- 3. this row half's partial gradients (plain stores: pp_adam_kernel reads them
  // after the launch boundary); each 16-column tile row is 64 contiguous bytes, the two
  // tiles of a row back to back
  PS_STAMP(24);
  float* const g = a.gpart + (long)h * a.gstride;
#pragma unroll
  for (int u = 0; u < UPW; ++u) {
    const int t = w + PS_NW * u;
    if (t >= NTK) break;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
      *reinterpret_cast<f32x4*>(g + (long)(16 * t + (lane & 15)) * PS_N + j0 + ct * 16 + 4 * (lane >> 4)) = dwa[u][ct];
  }
  if (tid < PS_CB) g[ps_g_b(K) + j0 + tid] = dba;
  if constexpr (LAST) {
    if (tid < PS_CB * PS_C) g[ps_g_wh(K) + (long)j0 * PS_C + tid] = dwh;
    if (cb == 0) {
      if (tid < PS_C) g[ps_g_bh(K) + tid] = dbh;
      l_loss = wave_sum(l_loss);
      l_corr = wave_sum(l_corr);
      if (lane == 0) { red[0][w] = l_loss; red[1][w] = l_corr; }
      __syncthreads();
      if (tid < 2) {
        float sum = 0.f;
        for (int q = 0; q < PS_NW; ++q) sum += red[tid][q];
        g[ps_g_met(K) + tid] = sum;
      }
    }
  }
  PS_STAMP(18);
}

template <bool FIRST, bool LAST>
__global__ void __launch_bounds__(PS_NT) pp_stage_kernel(PsArgs a) {
  __shared__ __attribute__((aligned(16))) char lds[PsLds<FIRST, LAST>::size];
  ps_body<FIRST, LAST>(a, blockIdx.x, lds);
}

// One GPU, every layer of an MLP pipeline a stage of ONE launch: stage s is workgroups
// [s PS_NB, (s+1) PS_NB), hand-offs through local inboxes (the same protocol as across
// ranks).  Every stage's workgroups must be resident at once (jdt_pp_chain_ok).
constexpr int PS_MAXCHAIN = 8;
struct PsChain {
  PsArgs st[PS_MAXCHAIN];
  int S;
  int adam_blk[PS_MAXCHAIN + 1];   // the AdamW launch: stage s owns blocks [adam_blk[s], adam_blk[s+1])
};

__global__ void __launch_bounds__(PS_NT) pp_chain_kernel(PsChain c) {
  __shared__ __attribute__((aligned(16))) char lds[PS_LDS_MAX];
  const int s = __builtin_amdgcn_readfirstlane(blockIdx.x / PS_NB), b = blockIdx.x % PS_NB;
  if (s == 0) ps_body<true, false>(c.st[0], b, lds);
  else if (s == c.S - 1) ps_body<false, true>(c.st[s], b, lds);
  else ps_body<false, false>(c.st[s], b, lds);
}

// AdamW of one stage over the whole chip, after pp_stage_kernel: g = half 0 + half 1
// (fixed order), scale 1 / n_mb; p / m / v, bf16 shadows; the last stage's head and
// metric fold; the last workgroup advances the optimizer step.
template <bool FIRST, bool LAST>
__device__ __forceinline__ void ps_adam_body(const PsArgs& a, const int blk, const int nblk, const int step) {
  constexpr int K = FIRST ? 784 : PS_N;
  const float t1 = (float)(step + 1);
  const float rbc1 = 1.f / (1.f - powf(a.b1, t1)), rbc2 = 1.f / (1.f - powf(a.b2, t1));
  auto adam = [&](float& p, float& m, float& v, float gr) {
    gr *= a.gscale;
    m = a.b1 * m + (1.f - a.b1) * gr;
    v = a.b2 * v + (1.f - a.b2) * gr * gr;
    p = p - a.lr * ((m * rbc1) * __builtin_amdgcn_rcpf(sqrtf(v * rbc2) + a.eps) + a.wd * p);
  };
  const float* g0 = a.gpart;
  const float* g1 = a.gpart + a.gstride;
  const long nw4 = (long)K * PS_N / 4;
  for (long q = (long)blk * blockDim.x + threadIdx.x; q < nw4; q += (long)nblk * blockDim.x) {
    const float4 x0 = reinterpret_cast<const float4*>(g0)[q], x1 = reinterpret_cast<const float4*>(g1)[q];
    float4 p = reinterpret_cast<const float4*>(a.p)[q], m = reinterpret_cast<const float4*>(a.m)[q],
           v = reinterpret_cast<const float4*>(a.v)[q];
    adam(p.x, m.x, v.x, x0.x + x1.x);
    adam(p.y, m.y, v.y, x0.y + x1.y);
    adam(p.z, m.z, v.z, x0.z + x1.z);
    adam(p.w, m.w, v.w, x0.w + x1.w);
    reinterpret_cast<float4*>(a.p)[q] = p;
    reinterpret_cast<float4*>(a.m)[q] = m;
    reinterpret_cast<float4*>(a.v)[q] = v;
    reinterpret_cast<uint2*>(a.sW)[q] = make_uint2((unsigned)f2bf(p.x) | ((unsigned)f2bf(p.y) << 16),
                                                   (unsigned)f2bf(p.z) | ((unsigned)f2bf(p.w) << 16));
  }
  if (blk == nblk - 1) {
    // the small leaves: b (+ W_h, b_h and the metric fold on the last stage)
    for (int j = threadIdx.x; j < PS_N; j += blockDim.x) {
      float p = a.pb[j], m = a.mbv[j], v = a.vb[j];
      adam(p, m, v, g0[ps_g_b(K) + j] + g1[ps_g_b(K) + j]);
      a.pb[j] = p; a.mbv[j] = m; a.vb[j] = v; a.sb[j] = f2bf(p);
    }
    if constexpr (LAST) {
      for (int j = threadIdx.x; j < PS_N * PS_C; j += blockDim.x) {
        float p = a.ph[j], m = a.mh[j], v = a.vh[j];
        adam(p, m, v, g0[ps_g_wh(K) + j] + g1[ps_g_wh(K) + j]);
        a.ph[j] = p; a.mh[j] = m; a.vh[j] = v; a.sh[j] = f2bf(p);
      }
      if (threadIdx.x < PS_C) {
        const int j = threadIdx.x;
        float p = a.phb[j], m = a.mhb[j], v = a.vhb[j];
        adam(p, m, v, g0[ps_g_bh(K) + j] + g1[ps_g_bh(K) + j]);
        a.phb[j] = p; a.mhb[j] = m; a.vhb[j] = v; a.shb[j] = f2bf(p);
      }
      if (threadIdx.x < 4) {
        // this step's loss sum / rows / correct / rows, folded into the running sums
        const int s = threadIdx.x;
        const float val = (s & 1) ? (float)(a.n_mb * a.mb)
                                  : g0[ps_g_met(K) + s / 2] + g1[ps_g_met(K) + s / 2];
        a.running[s] += a.mslot[s] + val;
        a.mslot[s] = 0.f;
      }
    }
  }
}

// the last workgroup of the launch to finish advances the optimizer step (every
// workgroup read it at its start)
__device__ __forceinline__ void ps_advance(int* step_p, unsigned* ticket, int step) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == gridDim.x - 1) {
      step_p[0] = step + 1;
      __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <bool FIRST, bool LAST>
__global__ void __launch_bounds__(256) pp_adam_kernel(PsArgs a) {
  const int step = a.step[0];
  ps_adam_body<FIRST, LAST>(a, blockIdx.x, gridDim.x, step);
  ps_advance(a.step, a.ticket, step);
}

// the chain's AdamW: stage s's leaves over blocks [adam_blk[s], adam_blk[s+1]); one step
// counter for the whole model
__global__ void __launch_bounds__(256) pp_adam_chain_kernel(PsChain c) {
  const int step = c.st[0].step[0];
  int s = 0;
  while (s + 1 < c.S && (int)blockIdx.x >= c.adam_blk[s + 1]) ++s;
  s = __builtin_amdgcn_readfirstlane(s);
  const int blk = blockIdx.x - c.adam_blk[s], nblk = c.adam_blk[s + 1] - c.adam_blk[s];
  if (s == 0) ps_adam_body<true, false>(c.st[0], blk, nblk, step);
  else if (s == c.S - 1) ps_adam_body<false, true>(c.st[s], blk, nblk, step);
  else ps_adam_body<false, false>(c.st[s], blk, nblk, step);
  ps_advance(c.st[0].step, c.st[0].ticket, step);
}

}  // namespace jdt
using namespace jdt;

JDT_API int jdt_pp_stage_args_size() { return (int)sizeof(PsArgs); }
// floats per row half of PsArgs::gpart for a stage whose layer input is `k` wide
JDT_API long jdt_pp_stage_gstride(int k) { return ps_g_size(k); }

// 1 if `nshare` ranks' stage launches (PS_NB workgroups each) can all be resident on
// this GPU at once (every wait of the launch is on a co-resident workgroup or a
// neighbour's launch), with half the device's workgroup slots to spare for the other
// ranks' kernels when the GPU is shared -- unless `spare` is 0: then every slot may hold
// a stage workgroup (8 stages x 32 workgroups on the 256 CUs, one per CU: the 8-stage
// test of the stage protocol on one GPU; the waits' timeouts bound a placement failure).
JDT_API int jdt_pp_stage_ok(int first, int last, int nshare, int spare) {
  int dev = 0, cus = 0, per = 0;
  if (nshare < 1 || hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  hipError_t e;
  if (first) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, pp_stage_kernel<true, false>, PS_NT, 0);
  else if (last) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, pp_stage_kernel<false, true>, PS_NT, 0);
  else e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, pp_stage_kernel<false, false>, PS_NT, 0);
  if (e != hipSuccess || per < 1) return 0;
  const long slots = (long)cus * per;
  return (long)nshare * PS_NB <= (nshare > 1 && spare ? slots / 2 : slots) ? 1 : 0;
}

// 1 if a chain of `S` stages (S x PS_NB workgroups of the one-GPU chain launch) can all be
// resident on this GPU at once
JDT_API int jdt_pp_chain_ok(int S) {
  int dev = 0, cus = 0, per = 0;
  if (S < 2 || S > PS_MAXCHAIN || hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, pp_chain_kernel, PS_NT, 0) != hipSuccess || per < 1)
    return 0;
  return (long)S * PS_NB <= (long)cus * per ? 1 : 0;
}
JDT_API int jdt_pp_chain_max() { return PS_MAXCHAIN; }

// One step of a one-GPU chain: args[0 .. S) are the stages' arguments (stage 0 takes the
// data, stage S - 1 carries the head; one step counter / ticket for all)
JDT_API int jdt_pp_chain(const PsArgs* args, int S, void* stream) {
  if (!args || S < 2 || S > PS_MAXCHAIN) return -2;
  PsChain c;
  c.S = S;
  c.adam_blk[0] = 0;
  for (int s = 0; s < S; ++s) {
    const PsArgs& a = args[s];
    const bool first = s == 0, last = s == S - 1;
    if ((a.mb != 32 && a.mb != 64) || a.n_mb * a.mb != PS_MAXROWS || a.K != (first ? 784 : PS_N) || !a.step ||
        a.step != args[0].step || !a.ticket || !a.ctr || !a.err || !a.gpart || a.gstride < ps_g_size(a.K))
      return -2;
    if (!first && (!a.in_mine || !a.flag_mine || !a.in_prev || !a.flag_prev || !a.w_prev || !a.wflag_prev)) return -2;
    if (!last && (!a.w_mine || !a.wflag_mine || !a.in_next || !a.flag_next)) return -2;
    if (first && (!a.X || !a.XT)) return -2;
    if (last && (!a.labels || !a.logits || !a.ph || !a.phb || !a.mslot || !a.running)) return -2;
    if (a.slot_bytes < (long)a.mb * PS_N * 4) return -2;
    c.st[s] = a;
    c.adam_blk[s + 1] = c.adam_blk[s] + (int)((((long)a.K * PS_N / 4) + 255) / 256);
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(pp_chain_kernel, dim3(S * PS_NB), dim3(PS_NT), 0, st, c);
  hipLaunchKernelGGL(pp_adam_chain_kernel, dim3(c.adam_blk[S]), dim3(256), 0, st, c);
  return HIP_LAUNCH_CHECK();
}

// One step of this stage (first: stage 0, last: the last stage; not both).
JDT_API int jdt_pp_stage(const PsArgs* args, int first, int last, void* stream) {
  const PsArgs& a = *args;
  if ((first && last) || (a.mb != 32 && a.mb != 64) || a.n_mb * a.mb != PS_MAXROWS || a.K != (first ? 784 : PS_N) ||
      !a.step || !a.ticket || !a.ctr || !a.err || !a.gpart || a.gstride < ps_g_size(a.K))
    return -2;
  if (!first && (!a.in_mine || !a.flag_mine || !a.in_prev || !a.flag_prev || !a.w_prev || !a.wflag_prev)) return -2;
  if (!last && (!a.w_mine || !a.wflag_mine)) return -2;
  if (!last && (!a.in_next || !a.flag_next)) return -2;
  if (first && (!a.X || !a.XT)) return -2;
  if (last && (!a.labels || !a.logits || !a.ph || !a.phb || !a.mslot || !a.running)) return -2;
  const long need = (long)a.mb * PS_N * 2 + (long)PS_N * a.mb * 2;
  if (a.slot_bytes < need) return -2;
  hipStream_t st = static_cast<hipStream_t>(stream);
  // the AdamW launch: one float4 of W per thread, every CU
  const int ga = (int)((((long)a.K * PS_N / 4) + 255) / 256);
  if (first) {
    hipLaunchKernelGGL((pp_stage_kernel<true, false>), dim3(PS_NB), dim3(PS_NT), 0, st, a);
    hipLaunchKernelGGL((pp_adam_kernel<true, false>), dim3(ga), dim3(256), 0, st, a);
  } else if (last) {
    hipLaunchKernelGGL((pp_stage_kernel<false, true>), dim3(PS_NB), dim3(PS_NT), 0, st, a);
    hipLaunchKernelGGL((pp_adam_kernel<false, true>), dim3(ga), dim3(256), 0, st, a);
  } else {
    hipLaunchKernelGGL((pp_stage_kernel<false, false>), dim3(PS_NB), dim3(PS_NT), 0, st, a);
    hipLaunchKernelGGL((pp_adam_kernel<false, false>), dim3(ga), dim3(256), 0, st, a);
  }
  return HIP_LAUNCH_CHECK();
}
