// Direct xGMI peer-to-peer collectives for the ranks of one MI355X node
// (native component N3).
//
// Why: the DP step all-reduces one 1.63 MB fp32 bucket (grads + 4 metric
// scalars, SURVEY X03+X04) while the whole fused compute step is ~20 us.  A
// ring all-reduce drives one xGMI link per GPU and pays 2(N-1) dependent hops;
// on a fully connected 8-GPU node every peer has its own link, so the
// two-shot direct algorithm below moves 2S/N bytes per link with exactly two
// synchronisation points:
//
//   phase 0  stage:  block b copies chunk b of every rank-slice of the local
//                    input into this rank's IPC buffer  data[par]
//   barrier A        (per block: "my chunk b is staged")
//   phase 1  reduce: block b sums chunk b of slice `rank` over all N peers'
//                    data buffers (all N remote loads in flight, fixed rank
//                    order, so every rank gets bit-identical sums) -> tmp[par]
//   barrier B        (per block: "my reduced chunk b is ready")
//   phase 2  gather: block b reads chunk b of slice q from peer q's tmp for all q
//                    (in flight together) and writes the output -- or, fused,
//                    applies AdamW to those elements and folds the metric
//                    slots into the running metrics (the step's optimizer and
//                    metrics fold run inside the collective: SURVEY K13/K14)
//
// Synchronisation is per block, never grid-wide: block b only touches chunk b
// of every slice, on every rank, so it only needs block b of the peers.  Flags
// are monotonically increasing per-block epochs written into the peers'
// signal pages with relaxed system-scope atomic stores, ordered after the data
// by vmcnt waits; every staging-buffer access is a system-scope sc0 sc1 buffer
// instruction (common.h "system-scope payload": write-through stores, coherent
// loads), so correctness does not depend on the MTYPE the importing GPU's IPC
// mapping inherits, and there is no L2 write-back/invalidate on the path.  The data and tmp
// buffers are double-buffered by the parity of a per-context call counter (every launch
// advances it once, XgSignal::calls), so a call may start staging while a slow peer
// still reads the previous call's buffers -- no trailing
// barrier.  Every spin has a wall-clock timeout (s_memrealtime, 100 MHz): a
// dead or desynchronised peer sets an error flag instead of hanging the GPU.
//
// Reduce-scatter (phases 0-1, result to the caller's shard) and all-gather
// (stage own shard, barrier, phase 2) reuse the same machinery for FSDP
// (SURVEY X05/X06).
#include "common.h"
#include "ipc_pool.h"

#include <cstring>

namespace jdt {

constexpr int XG_MAX_RANKS = 8;
constexpr int XG_MAX_BLOCKS = 96;
constexpr int XG_THREADS = 256;

struct XgSignal {
  unsigned flag[2][XG_MAX_BLOCKS][XG_MAX_RANKS];  // [barrier][block][src rank], written by the peers
  unsigned epoch[XG_MAX_BLOCKS];                   // calls completed by each local block
  int err;                                         // 1 = a barrier timed out
  // the first timeout's site (kernel * 2 + barrier), block, awaited epoch, silent peer
  unsigned errinfo[4];
  // local only (never touched by peers): every launch on this context advances `calls`
  // once (its last block, by `call_ticket`); the parity of `calls` selects the
  // data / tmp half of every unstaged call.  Per-block epoch parity cannot: a block that
  // sat out the previous call (that call had fewer blocks) keeps a stale parity and
  // would write the half a slow peer may still be reading after a single-barrier call
  // (one-shot all-reduce, segmented all-gather / reduce-scatter).
  unsigned calls;
  unsigned call_ticket;
};

// Read the call counter (thread 0; every block reads it before the last block's ticket).
__device__ __forceinline__ unsigned xg_calls(XgSignal* me) {
  return __hip_atomic_load(&me->calls, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// End of a block's part of the call: the last block advances the call counter.
__device__ __forceinline__ void xg_call_done(XgSignal* me) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(&me->call_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == gridDim.x - 1) {
      __hip_atomic_store(&me->call_ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(&me->calls, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

struct XgPeers {
  float* data[XG_MAX_RANKS];  // 2 halves of cap floats each (epoch parity)
  float* tmp[XG_MAX_RANKS];
  XgSignal* sig[XG_MAX_RANKS];
};

struct XgAdam {  // fused AdamW + metrics fold over the reduced buffer (phase 2)
  float* p;
  float* m;
  float* v;
  bf16_t* shadow;
  long n_params;   // AdamW range [0, n_params), multiple of 4
  float* running;  // running[j] += reduced[n_params + j], j < n_metrics
  int n_metrics;
  float lr, b1, b2, eps, wd, grad_scale;
  int* step;
  unsigned* ticket;
  float* zero;     // zero these indices of this buffer after reading (the grad bucket) or null
  // 1: do not advance *step at the end (one of several per-bucket calls of a step that
  // overlap the backward, parallel/pipeline.py; the step's last call advances it)
  int hold;
  // 1: p / m / v / shadow stored write-through (agent-scope sc1): not left dirty in this
  // XCD's L2 for the kernel boundary to write back (ops/csrc/mlp_fused.hip Mlp2Args::wt)
  int wt;
};

enum { XG_ALLREDUCE = 0, XG_REDUCE_SCATTER = 1, XG_ALL_GATHER = 2 };

__device__ __forceinline__ unsigned long long xg_now() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ float4 add4(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

// Per-block barrier across the W ranks.  Thread q < W signals peer q and waits for
// peer q's signal.  Every wave's payload stores are sc0 sc1 (write-through at
// system scope) and are drained (vmcnt) before the workgroup barrier that
// precedes the flag store; flags are relaxed system-scope atomic stores / loads,
// and all payload loads after the wait are sc0 sc1 (common.h), so no cache
// maintenance instruction is needed.  (A release/acquire pair would lower to
// a write-back / invalidate of the whole L2 -- per wave, and per spin iteration
// on the acquire side: measured ~70 us for a 1 MB all-reduce, tools/bench_comm.py.)
// site: kernel id (XG_SITE_*) * 2 + which, recorded with the first timeout (errinfo)
enum { XG_SITE_TWOSHOT = 1, XG_SITE_ONESHOT = 2, XG_SITE_SEG = 3, XG_SITE_FSDP = 4 };
__device__ void xg_barrier(const XgPeers& P, int rank, int W, int which, unsigned epoch, long long timeout,
                           int kernel = 0) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int b = blockIdx.x;
  if (threadIdx.x < W) {
    const int q = threadIdx.x;
    __hip_atomic_store(&P.sig[q]->flag[which][b][rank], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    XgSignal* me = P.sig[rank];
    const unsigned long long t0 = xg_now();
    while ((int)(__hip_atomic_load(&me->flag[which][b][q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
      if ((long long)(xg_now() - t0) > timeout) {
        int zero = 0;
        if (__hip_atomic_compare_exchange_strong(&me->err, &zero, 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_SYSTEM)) {
          me->errinfo[0] = (unsigned)(kernel * 2 + which);
          me->errinfo[1] = (unsigned)b;
          me->errinfo[2] = epoch;
          me->errinfo[3] = (unsigned)q;
        }
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

__device__ __forceinline__ float4 load_guard(const float* src, long e, long n) {
  if (e + 3 < n) return *reinterpret_cast<const float4*>(src + e);
  float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e < n) x.x = src[e];
  if (e + 1 < n) x.y = src[e + 1];
  if (e + 2 < n) x.z = src[e + 2];
  return x;
}

__device__ __forceinline__ void store_guard(float* dst, long e, long n, float4 x) {
  if (e + 3 < n) { *reinterpret_cast<float4*>(dst + e) = x; return; }
  if (e < n) dst[e] = x.x;
  if (e + 1 < n) dst[e + 1] = x.y;
  if (e + 2 < n) dst[e + 2] = x.z;
}

typedef __attribute__((address_space(1))) unsigned long long xg_gu64;
__device__ __forceinline__ void wt_store8(void* p, unsigned long long x) {
  __hip_atomic_store((xg_gu64*)p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // global_store ... sc1
}
__device__ __forceinline__ void wt_store16(float* p, float4 x) {
  wt_store8(p, (unsigned long long)__float_as_uint(x.x) | ((unsigned long long)__float_as_uint(x.y) << 32));
  wt_store8(p + 2, (unsigned long long)__float_as_uint(x.z) | ((unsigned long long)__float_as_uint(x.w) << 32));
}
// the fused AdamW's stores of element group e: p, m, v and the bf16 shadow
__device__ __forceinline__ void adam_store(const XgAdam& A, long e, float4 pp, float4 mm, float4 vv) {
  unsigned long long sh = 0ull;
  if (A.shadow)
    sh = (unsigned long long)((unsigned)f2bf(pp.x) | ((unsigned)f2bf(pp.y) << 16)) |
         ((unsigned long long)((unsigned)f2bf(pp.z) | ((unsigned)f2bf(pp.w) << 16)) << 32);
  if (A.wt) {
    wt_store16(A.p + e, pp); wt_store16(A.m + e, mm); wt_store16(A.v + e, vv);
    if (A.shadow) wt_store8(A.shadow + e, sh);
  } else {
    *reinterpret_cast<float4*>(A.p + e) = pp;
    *reinterpret_cast<float4*>(A.m + e) = mm;
    *reinterpret_cast<float4*>(A.v + e) = vv;
    if (A.shadow) *reinterpret_cast<unsigned long long*>(A.shadow + e) = sh;
  }
}

__device__ __forceinline__ float4 adam4(const XgAdam& A, long e, float4 g, float rbc1, float rbc2) {
  float4 pp = *reinterpret_cast<float4*>(A.p + e);
  float4 mm = *reinterpret_cast<float4*>(A.m + e);
  float4 vv = *reinterpret_cast<float4*>(A.v + e);
  float* pe = &pp.x; float* me = &mm.x; float* ve = &vv.x; const float* ge = &g.x;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float gr = ge[k] * A.grad_scale;
    me[k] = A.b1 * me[k] + (1.f - A.b1) * gr;
    ve[k] = A.b2 * ve[k] + (1.f - A.b2) * gr * gr;
    pe[k] -= A.lr * ((me[k] * rbc1) / (sqrtf(ve[k] * rbc2) + A.eps) + A.wd * pe[k]);
  }
  adam_store(A, e, pp, mm, vv);
  return pp;
}

// Caller layout: rank q's part of the full vector is [q*s, q*s + s) (s % 4 == 0),
// valid up to n.  Kernel layout in the IPC buffers: [q*slice, q*slice + s) with
// slice = G * chunk >= s, block b owning positions [b*chunk, (b+1)*chunk).
// ALLREDUCE:      in[n] -> out[n] (or fused AdamW + metrics fold)
// REDUCE_SCATTER: in[n] -> out[0, s) = reduced part `rank`
// ALL_GATHER:     in[0, s) = part `rank` -> out[n]
// staged (ALLREDUCE + fused AdamW only): the producer kernel of the step (mlp2_bwd /
// md_bwd mode 0) already wrote this rank's gradient bucket straight into its data
// buffer, identity layout (slice == s), in the half selected by the parity of the
// optimizer step counter A.step -- which every block reads here before the last
// block's ticket advances it -- so phase 0 (a full-buffer copy) is skipped.
// Latency structure: a thread owns nit = ceil(nv / 256) float4 positions of its block's
// chunk (1 at W = 8, 2-3 at W = 2..4 for the DP bucket).  Every phase issues ALL of a
// thread's loads for up to XG_MI(W) positions before its first store (vmcnt counts loads
// and stores together on gfx9, so a load behind a store waits for that store), and the
// fused AdamW state (p, m, v -- local, unaffected by the collective) is loaded before
// barrier B, so it arrives while the block waits for its peers.
template <int W> struct XgMi { static constexpr int v = W <= 2 ? 4 : (W <= 4 ? 2 : 1); };

__device__ __forceinline__ float4 adam4_pre(const XgAdam& A, long e, float4 g, float4 pp, float4 mm, float4 vv,
                                            float rbc1, float rbc2) {
  float* pe = &pp.x; float* me = &mm.x; float* ve = &vv.x; const float* ge = &g.x;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float gr = ge[k] * A.grad_scale;
    me[k] = A.b1 * me[k] + (1.f - A.b1) * gr;
    ve[k] = A.b2 * ve[k] + (1.f - A.b2) * gr * gr;
    pe[k] -= A.lr * ((me[k] * rbc1) / (sqrtf(ve[k] * rbc2) + A.eps) + A.wd * pe[k]);
  }
  adam_store(A, e, pp, mm, vv);
  return pp;
}

template <int W, int OP>
__global__ void __launch_bounds__(XG_THREADS) xg_kernel(XgPeers P, int rank, long cap, const float* in, float* out,
                                                        long n, long s, long slice,
                                                        long chunk, XgAdam A, int fuse, long long timeout,
                                                        int staged) {
  constexpr int MI = XgMi<W>::v;
  __shared__ unsigned s_epoch, s_calls;
  const int b = blockIdx.x;
  XgSignal* me = P.sig[rank];
  if (threadIdx.x == 0) {
    s_epoch = me->epoch[b] + 1u;
    s_calls = xg_calls(me);
  }
  __syncthreads();
  const unsigned epoch = s_epoch;
  const long half = (long)((staged ? (unsigned)A.step[0] : s_calls) & 1u) * cap;
  const long base = (long)b * chunk;
  const int nv = (int)(chunk >> 2);
  const int nit = (nv + XG_THREADS - 1) / XG_THREADS;
  const long own_n = (n - rank * s < s) ? n - rank * s : s;  // valid length of this rank's part
  const unsigned long long bytes = (unsigned long long)cap * 2ull * sizeof(float);
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  // every access to an IPC buffer (own or peer) is a system-scope sc0 sc1 access (common.h)
  __amdgpu_buffer_rsrc_t rdata[W], rtmp[W];
#pragma unroll
  for (int q = 0; q < W; ++q) {
    rdata[q] = sys_rsrc(P.data[q], bytes);
    rtmp[q] = sys_rsrc(P.tmp[q], bytes);
  }
  const __amdgpu_buffer_rsrc_t my_data = sys_rsrc(P.data[rank], bytes), my_tmp = sys_rsrc(P.tmp[rank], bytes);

  if (OP != XG_ALL_GATHER) {
    // phase 0: stage chunk b of every part of the local input (write-through stores):
    // all (part, position) loads of a round first, then the stores
    if (!staged) {
      for (int t0 = 0; t0 < W * nit; t0 += MI) {
        float4 x[MI];
        long d[MI];
#pragma unroll
        for (int u = 0; u < MI; ++u) {
          const int t = t0 + u, q = t / nit, i = threadIdx.x + (t % nit) * XG_THREADS;
          const long j = base + 4 * (long)i;
          x[u] = z4;
          d[u] = -1;
          if (t < W * nit && i < nv) {
            d[u] = half + q * slice + j;
            if (j < s) x[u] = load_guard(in, q * s + j, n);
          }
        }
#pragma unroll
        for (int u = 0; u < MI; ++u)
          if (d[u] >= 0) sys_store4(my_data, d[u], x[u]);
      }
    }
    xg_barrier(P, rank, W, 0, epoch, timeout, XG_SITE_TWOSHOT);
    // phase 1: reduce chunk b of part `rank` over the peers (W x MI loads in flight,
    // fixed rank order -> every rank computes bit-identical sums)
    for (int i0 = 0; i0 < nit; i0 += MI) {
      float4 v[MI][W];
#pragma unroll
      for (int u = 0; u < MI; ++u) {
        const int i = min(threadIdx.x + (i0 + u) * XG_THREADS, nv - 1);   // clamped: unconditional loads
        const long e = rank * slice + base + 4 * (long)i;
#pragma unroll
        for (int q = 0; q < W; ++q) v[u][q] = sys_load4(rdata[q], half + e);
      }
#pragma unroll
      for (int u = 0; u < MI; ++u) {
        const int i = threadIdx.x + (i0 + u) * XG_THREADS;
        if (i0 + u >= nit || i >= nv) continue;
        const long j = base + 4 * (long)i;
        float4 acc = v[u][0];
#pragma unroll
        for (int q = 1; q < W; ++q) acc = add4(acc, v[u][q]);
        if (OP == XG_REDUCE_SCATTER) store_guard(out, j, own_n, acc);
        else sys_store4(my_tmp, half + rank * slice + j, acc);
      }
    }
    if (OP == XG_REDUCE_SCATTER) {
      if (threadIdx.x == 0) me->epoch[b] = epoch;
      xg_call_done(me);
      return;
    }
  } else {
    // all-gather phase 0: stage chunk b of this rank's part into its tmp slice
    for (int i = threadIdx.x; i < nv; i += XG_THREADS) {
      const long j = base + 4 * i;
      const float4 x = j < s ? load_guard(in, j, own_n) : z4;
      sys_store4(my_tmp, half + rank * slice + j, x);
    }
  }
  float rbc1 = 1.f, rbc2 = 1.f;
  if (fuse) {
    const int t = A.step[0] + 1;
    rbc1 = 1.f / (1.f - powf(A.b1, (float)t));
    rbc2 = 1.f / (1.f - powf(A.b2, (float)t));
  }
  // phase 2: gather chunk b of every part (all W x MI loads in flight per thread).  Fused,
  // W <= 4: the AdamW state of the first round's elements is loaded before barrier B (at
  // W > 4 its 3W float4 registers would halve the occupancy, and ranks sharing one GPU
  // need every rank's grid resident at once for the barriers)
  constexpr bool PRE = W <= 4;
  constexpr int WP = PRE ? W : 1;
  const bool pre = PRE && fuse && A.n_params >= 4;
  const long pcl = pre ? A.n_params - 4 : 0;
  float4 sp[MI][WP], sm[MI][WP], sv[MI][WP];
  for (int i0 = 0; i0 < nit; i0 += MI) {
    if (pre) {
#pragma unroll
      for (int u = 0; u < MI; ++u) {
        const long j = base + 4 * (long)min(threadIdx.x + (i0 + u) * XG_THREADS, nv - 1);
#pragma unroll
        for (int q = 0; q < WP; ++q) {
          const long e = min((long)q * s + j, pcl);
          sp[u][q] = *reinterpret_cast<const float4*>(A.p + e);
          sm[u][q] = *reinterpret_cast<const float4*>(A.m + e);
          sv[u][q] = *reinterpret_cast<const float4*>(A.v + e);
        }
      }
    }
    if (i0 == 0) xg_barrier(P, rank, W, 1, epoch, timeout, XG_SITE_TWOSHOT);
    float4 r[MI][W];
#pragma unroll
    for (int u = 0; u < MI; ++u) {
      const long j = base + 4 * (long)min(threadIdx.x + (i0 + u) * XG_THREADS, nv - 1);
#pragma unroll
      for (int q = 0; q < W; ++q) r[u][q] = sys_load4(rtmp[q], half + q * slice + j);
    }
#pragma unroll
    for (int u = 0; u < MI; ++u) {
      const int i = threadIdx.x + (i0 + u) * XG_THREADS;
      const long j = base + 4 * (long)i;
      if (i0 + u >= nit || i >= nv || j >= s) continue;
#pragma unroll
      for (int q = 0; q < W; ++q) {
        const long e = q * s + j;
        if (!fuse) {
          store_guard(out, e, n, r[u][q]);
        } else if (e < n) {
          if (e < A.n_params) {
            if (PRE && pre) adam4_pre(A, e, r[u][q], sp[u][q % WP], sm[u][q % WP], sv[u][q % WP], rbc1, rbc2);
            else adam4(A, e, r[u][q], rbc1, rbc2);
          } else {
            const float* rv = &r[u][q].x;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const long mj = e + k - A.n_params;
              if (mj < A.n_metrics && e + k < n) A.running[mj] += rv[k];
            }
          }
          if (A.zero) store_guard(A.zero, e, n, z4);
        }
      }
    }
  }
  if (nit == 0) xg_barrier(P, rank, W, 1, epoch, timeout, XG_SITE_TWOSHOT);
  if (threadIdx.x == 0) me->epoch[b] = epoch;
  if (fuse && A.step && !A.hold) {
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned t = atomicAdd(A.ticket, 1u);
      if (t == gridDim.x - 1) {
        A.step[0] = A.step[0] + 1;
        __hip_atomic_store(A.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  xg_call_done(me);
}

// ---------------------------------------------------------------------------
// One-shot all-reduce for small messages (<= g_oneshot_bytes, 256 KiB by default,
// SURVEY 5.8 (b)): block b stages chunk b of the WHOLE input, one barrier, then
// reads chunk b from every peer (all W loads in flight) and sums in rank order --
// the same order as the two-shot kernel, so results are bit-identical -- one
// synchronisation point instead of two and no second (gather) pass, which is the
// cost that matters at latency-bound sizes.  Same double-buffered data halves,
// epochs and per-block discipline as xg_kernel (a block only writes and reads
// chunk b of a call; kernels of one stream do not overlap), fused AdamW + metrics.
template <int W>
__global__ void __launch_bounds__(XG_THREADS) xg_oneshot_kernel(XgPeers P, int rank, long cap, const float* in,
                                                                float* out, long n, long chunk, XgAdam A, int fuse,
                                                                long long timeout) {
  __shared__ unsigned s_epoch, s_calls;
  const int b = blockIdx.x;
  XgSignal* me = P.sig[rank];
  if (threadIdx.x == 0) {
    s_epoch = me->epoch[b] + 1u;
    s_calls = xg_calls(me);
  }
  __syncthreads();
  const unsigned epoch = s_epoch;
  const long half = (long)(s_calls & 1u) * cap;
  const long base = (long)b * chunk;
  const int nv = (int)(chunk >> 2);
  const unsigned long long bytes = (unsigned long long)cap * 2ull * sizeof(float);
  __amdgpu_buffer_rsrc_t rdata[W];
#pragma unroll
  for (int q = 0; q < W; ++q) rdata[q] = sys_rsrc(P.data[q], bytes);
  const __amdgpu_buffer_rsrc_t my_data = sys_rsrc(P.data[rank], bytes);
  constexpr int MI = XgMi<W>::v;   // positions per thread per round (xg_kernel's latency structure)
  const int nit = (nv + XG_THREADS - 1) / XG_THREADS;
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int i0 = 0; i0 < nit; i0 += MI) {
    float4 x[MI];
#pragma unroll
    for (int u = 0; u < MI; ++u) {
      const long j = base + 4 * (long)(threadIdx.x + (i0 + u) * XG_THREADS);
      x[u] = (i0 + u < nit && j < base + chunk && j < n) ? load_guard(in, j, n) : z4;
    }
#pragma unroll
    for (int u = 0; u < MI; ++u) {
      const long j = base + 4 * (long)(threadIdx.x + (i0 + u) * XG_THREADS);
      if (i0 + u < nit && j < base + chunk) sys_store4(my_data, half + j, x[u]);
    }
  }
  float rbc1 = 1.f, rbc2 = 1.f;
  if (fuse) {
    const int t = A.step[0] + 1;
    rbc1 = 1.f / (1.f - powf(A.b1, (float)t));
    rbc2 = 1.f / (1.f - powf(A.b2, (float)t));
  }
  const bool pre = W <= 4 && fuse && A.n_params >= 4;   // register budget as in xg_kernel
  const long pcl = pre ? A.n_params - 4 : 0;
  for (int i0 = 0; i0 < nit; i0 += MI) {
    float4 sp[MI], sm[MI], sv[MI];
    if (pre) {   // AdamW state (local) of this round: in flight across the barrier
#pragma unroll
      for (int u = 0; u < MI; ++u) {
        const long e = min(base + 4 * (long)min(threadIdx.x + (i0 + u) * XG_THREADS, nv - 1), pcl);
        sp[u] = *reinterpret_cast<const float4*>(A.p + e);
        sm[u] = *reinterpret_cast<const float4*>(A.m + e);
        sv[u] = *reinterpret_cast<const float4*>(A.v + e);
      }
    }
    if (i0 == 0) xg_barrier(P, rank, W, 0, epoch, timeout, XG_SITE_ONESHOT);
    float4 v[MI][W];
#pragma unroll
    for (int u = 0; u < MI; ++u) {
      const long j = base + 4 * (long)min(threadIdx.x + (i0 + u) * XG_THREADS, nv - 1);
#pragma unroll
      for (int q = 0; q < W; ++q) v[u][q] = sys_load4(rdata[q], half + j);
    }
#pragma unroll
    for (int u = 0; u < MI; ++u) {
      const int i = threadIdx.x + (i0 + u) * XG_THREADS;
      const long j = base + 4 * (long)i;
      if (i0 + u >= nit || i >= nv || j >= n) continue;
      float4 acc = v[u][0];
#pragma unroll
      for (int q = 1; q < W; ++q) acc = add4(acc, v[u][q]);
      if (!fuse) {
        store_guard(out, j, n, acc);
      } else {
        if (j < A.n_params) {
          if (pre) adam4_pre(A, j, acc, sp[u], sm[u], sv[u], rbc1, rbc2);
          else adam4(A, j, acc, rbc1, rbc2);
        } else {
          const float* rv = &acc.x;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const long mj = j + k - A.n_params;
            if (mj < A.n_metrics && j + k < n) A.running[mj] += rv[k];
          }
        }
        if (A.zero) store_guard(A.zero, j, n, z4);
      }
    }
  }
  if (threadIdx.x == 0) me->epoch[b] = epoch;
  if (fuse && A.step && !A.hold) {
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned t = atomicAdd(A.ticket, 1u);
      if (t == gridDim.x - 1) {
        A.step[0] = A.step[0] + 1;
        __hip_atomic_store(A.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  xg_call_done(me);
}

// ---------------------------------------------------------------------------
// Segmented all-gather / reduce-scatter: several tensors ("segments", e.g. the
// dim-0-sharded leaves of an FSDP model) in ONE launch, each gathered straight
// into / scattered straight out of its own full-tensor layout.  Rank q's part of
// segment k is full_k[q*s_k, (q+1)*s_k) (words, valid up to nfull_k); in the IPC
// buffers rank q's parts of all segments are packed at [q*slice + off_k, +s_k).
// Words are 4 bytes, so bf16 shadow shards and fp32 grads use the same kernel.
constexpr int XG_MAX_SEGS = 16;

struct XgSeg {
  float* full;
  float* part;
  long s;      // part length (words, multiple of 4)
  long off;    // packed offset (words, multiple of 4)
  long nfull;  // valid words of full
  // reduce-scatter only: an ALL-REDUCE segment riding in the same launch -- every
  // rank contributes its whole full[0, s) as each peer's part, so part[0, s) receives
  // the sum over ranks (FSDP: the replicated leaves' grads + metric slots, which
  // otherwise cost a collective launch of their own); never accumulated
  long bcast;
  // 2-D (dim-1) shards: rows > 1 -> part is [rows][s / rows] contiguous and rank q's
  // part of full is the column block full[r * ld + q * qoff + c] (a square weight is
  // sharded along its LAST dim by the reference rule, param_sharding.py:82-118);
  // rows <= 1: the 1-D layout above (rank q's part = full[q * s, (q + 1) * s))
  long rows, ld, qoff;
};

// word index in `full` of word jj of rank q's part
__device__ __forceinline__ long seg_full_index(const XgSeg& g, int q, long jj) {
  if (g.rows <= 1) return (g.bcast ? 0 : (long)q * g.s) + jj;
  const long w = g.s / g.rows;
  const long r = jj / w;
  return r * g.ld + (long)q * g.qoff + (jj - r * w);
}

struct XgSegs {
  XgSeg seg[XG_MAX_SEGS];
  int n;
  long S;  // sum of s
};

__device__ __forceinline__ int xg_find(const XgSegs& S, long j) {
  int k = 0;
  for (int t = 1; t < S.n; ++t)
    if (j >= S.seg[t].off) k = t;
  return k;
}

template <int W, int OP>
__global__ void __launch_bounds__(XG_THREADS) xg_seg_kernel(XgPeers P, int rank, long cap, XgSegs S, long slice,
                                                            long chunk, int accumulate, long long timeout) {
  __shared__ unsigned s_epoch, s_calls;
  const int b = blockIdx.x;
  XgSignal* me = P.sig[rank];
  if (threadIdx.x == 0) {
    s_epoch = me->epoch[b] + 1u;
    s_calls = xg_calls(me);
  }
  __syncthreads();
  const unsigned epoch = s_epoch;
  const long half = (long)(s_calls & 1u) * cap;
  const long base = (long)b * chunk;
  const int nv = (int)(chunk >> 2);
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  const unsigned long long bytes = (unsigned long long)cap * 2ull * sizeof(float);

  if (OP == XG_REDUCE_SCATTER) {
    const __amdgpu_buffer_rsrc_t my_data = sys_rsrc(P.data[rank], bytes);
    for (int q = 0; q < W; ++q) {
      for (int i = threadIdx.x; i < nv; i += XG_THREADS) {
        const long j = base + 4 * i;
        float4 x = z4;
        if (j < S.S) {
          const XgSeg& g = S.seg[xg_find(S, j)];
          x = load_guard(g.full, seg_full_index(g, q, j - g.off), g.nfull);
        }
        sys_store4(my_data, half + q * slice + j, x);
      }
    }
    xg_barrier(P, rank, W, 0, epoch, timeout, XG_SITE_SEG);
    __amdgpu_buffer_rsrc_t rdata[W];
#pragma unroll
    for (int q = 0; q < W; ++q) rdata[q] = sys_rsrc(P.data[q], bytes);
    for (int i = threadIdx.x; i < nv; i += XG_THREADS) {
      const long j = base + 4 * i;
      if (j >= S.S) break;
      float4 v[W];
#pragma unroll
      for (int q = 0; q < W; ++q) v[q] = sys_load4(rdata[q], half + rank * slice + j);
      float4 acc = v[0];
#pragma unroll
      for (int q = 1; q < W; ++q) acc = add4(acc, v[q]);
      const XgSeg& g = S.seg[xg_find(S, j)];
      const long lim = g.bcast ? g.nfull : ((g.nfull - rank * g.s < g.s) ? g.nfull - rank * g.s : g.s);
      if (accumulate && !g.bcast) acc = add4(acc, load_guard(g.part, j - g.off, lim));
      store_guard(g.part, j - g.off, lim, acc);
    }
  } else {
    const __amdgpu_buffer_rsrc_t my_tmp = sys_rsrc(P.tmp[rank], bytes);
    for (int i = threadIdx.x; i < nv; i += XG_THREADS) {
      const long j = base + 4 * i;
      float4 x = z4;
      if (j < S.S) {
        const XgSeg& g = S.seg[xg_find(S, j)];
        const long lim = (g.nfull - rank * g.s < g.s) ? g.nfull - rank * g.s : g.s;
        x = load_guard(g.part, j - g.off, lim);
      }
      sys_store4(my_tmp, half + rank * slice + j, x);
    }
    xg_barrier(P, rank, W, 1, epoch, timeout, XG_SITE_SEG);
    __amdgpu_buffer_rsrc_t rtmp[W];
#pragma unroll
    for (int q = 0; q < W; ++q) rtmp[q] = sys_rsrc(P.tmp[q], bytes);
    for (int i = threadIdx.x; i < nv; i += XG_THREADS) {
      const long j = base + 4 * i;
      if (j >= S.S) break;
      float4 r[W];
#pragma unroll
      for (int q = 0; q < W; ++q) r[q] = sys_load4(rtmp[q], half + q * slice + j);
      const XgSeg& g = S.seg[xg_find(S, j)];
#pragma unroll
      for (int q = 0; q < W; ++q) store_guard(g.full, seg_full_index(g, q, j - g.off), g.nfull, r[q]);
    }
  }
  if (threadIdx.x == 0) me->epoch[b] = epoch;
  xg_call_done(me);
}


// ---------------------------------------------------------------------------
// The whole FSDP (ZeRO-3) communication of a step in ONE launch, for the fused
// engines' plain-stored full gradients:
//   phase 0  stage every peer part of every segment's full fp32 gradient
//   barrier
//   phase 1  reduce this rank's part (rank-ordered sum) and, per element:
//            sharded leaf  -> AdamW on the LOCAL shard (fp32 master, m, v, bf16 local
//                             shadow), the new bf16 value into tmp for the peers;
//            replicated    -> (an all-reduce segment) AdamW on every rank, bf16 straight
//                             into the full shadow;
//            metric slots  -> running metrics += sum, slots zeroed
//   barrier
//   phase 2  gather every peer's updated bf16 shard into the full bf16 shadow the
//            next step's forward reads (the all-gather of the NEXT step, done now)
// so an N > 1 FSDP step is the fused forward, the fused backward and this kernel --
// the separate gather, reduce-scatter, AdamW and metrics-fold launches are gone.
// Geometry as xg_seg_kernel (segments packed by `off`, `bcast` = all-reduce
// segment); bf16 values travel in the tmp buffer at bf16 index 2*half + q*slice + j.
enum { XF_SHARD = 0, XF_REPL = 1, XF_METRIC = 2 };
struct XgFsdp {
  XgAdam A;                        // p / m / v / shadow = the LOCAL flat buffers; running = metrics
  const float* grad;               // local grad base: a part's local offset = part - grad
  int kind[XG_MAX_SEGS];
  bf16_t* full_shadow[XG_MAX_SEGS];  // bf16 full leaf (gather / replicated target)
  // diagnostic (tools/stamp_xg_fsdp.py): per block s_memrealtime at the phase edges
  // [G][8]: start, stage stored, barrier A, reduce + AdamW, barrier B, gather, end
  unsigned long long* stamps;
  // 1: the step's producer kernel (mlp2_bwd / md_bwd mode 0 with a common.h StageMap)
  // already wrote every peer part of every segment into this rank's data buffer, in the
  // half of the optimizer step's parity (A.step, read by every block before the last
  // block's ticket advances it) -- phase 0 is skipped, as in xg_kernel's staged mode
  int staged;
};

#define XF_STAMP(i)                                                                            \
  do {                                                                                         \
    if (F.stamps && threadIdx.x == 0) F.stamps[(long)blockIdx.x * 8 + (i)] = xg_now();       \
  } while (0)

__device__ __forceinline__ void sys_store8(__amdgpu_buffer_rsrc_t r, long byte_off, uint2 x) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(__attribute__((ext_vector_type(2))) unsigned, x), r,
                                        (int)byte_off, 0, CPOL_SYS);
}
__device__ __forceinline__ uint2 sys_load8(__amdgpu_buffer_rsrc_t r, long byte_off) {
  return __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(r, (int)byte_off, 0, CPOL_SYS));
}

template <int W>
__global__ void __launch_bounds__(XG_THREADS) xg_fsdp_kernel(XgPeers P, int rank, long cap, XgSegs S, XgFsdp F,
                                                             long slice, long chunk, long long timeout) {
  __shared__ unsigned s_epoch, s_calls;
  const int b = blockIdx.x;
  XgSignal* me = P.sig[rank];
  if (threadIdx.x == 0) {
    s_epoch = me->epoch[b] + 1u;
    s_calls = xg_calls(me);
  }
  __syncthreads();
  const unsigned epoch = s_epoch;
  const XgAdam& A = F.A;
  const long half = (long)((F.staged ? (unsigned)A.step[0] : s_calls) & 1u) * cap;
  const long base = (long)b * chunk;
  const int nv = (int)(chunk >> 2);
  const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
  const unsigned long long bytes = (unsigned long long)cap * 2ull * sizeof(float);
  XF_STAMP(0);

  // Latency structure as xg_kernel: a thread's loads of a round are all issued before
  // its first store (M0 / MI positions per round), the sharded AdamW state of the first
  // round is loaded before barrier A.
  constexpr int M0 = 8, MI = XgMi<W>::v;
  const int nit = (nv + XG_THREADS - 1) / XG_THREADS;

  // phase 0: stage (skipped when the producer staged the bucket)
  if (!F.staged) {
    const __amdgpu_buffer_rsrc_t my_data = sys_rsrc(P.data[rank], bytes);
    for (int t0 = 0; t0 < W * nit; t0 += M0) {
      float4 x[M0];
      long d[M0];
#pragma unroll
      for (int u = 0; u < M0; ++u) {
        const int t = t0 + u, q = t / nit, i = threadIdx.x + (t % nit) * XG_THREADS;
        const long j = base + 4 * (long)i;
        x[u] = z4;
        d[u] = -1;
        if (t < W * nit && i < nv) {
          d[u] = half + q * slice + j;
          if (j < S.S) {
            const XgSeg& g = S.seg[xg_find(S, j)];
            x[u] = load_guard(g.full, seg_full_index(g, q, j - g.off), g.nfull);
          }
        }
      }
#pragma unroll
      for (int u = 0; u < M0; ++u)
        if (d[u] >= 0) sys_store4(my_data, d[u], x[u]);
    }
  }
  if (F.stamps) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); XF_STAMP(1); }

  // phase 1: reduce own part, optimizer, publish the new bf16 shard
  float rbc1, rbc2;
  {
    const int t = A.step[0] + 1;
    rbc1 = 1.f / (1.f - powf(A.b1, (float)t));
    rbc2 = 1.f / (1.f - powf(A.b2, (float)t));
  }
  {
    __amdgpu_buffer_rsrc_t rdata[W];
#pragma unroll
    for (int q = 0; q < W; ++q) rdata[q] = sys_rsrc(P.data[q], bytes);
    const __amdgpu_buffer_rsrc_t my_tmp = sys_rsrc(P.tmp[rank], bytes);
    for (int i0 = 0; i0 < nit; i0 += MI) {
      // this round's positions: segment, local offset, and (aligned whole groups) the
      // AdamW state -- local, so it is loaded while the block waits at barrier A
      int kk[MI];
      long jjv[MI], lov[MI], limv[MI];
      bool live[MI], fast[MI];
      float4 sp[MI], sm[MI], sv[MI];
#pragma unroll
      for (int u = 0; u < MI; ++u) {
        const int i = threadIdx.x + (i0 + u) * XG_THREADS;
        const long j = base + 4 * (long)i;
        live[u] = i0 + u < nit && i < nv && j < S.S;
        const int k = live[u] ? xg_find(S, j) : 0;
        const XgSeg& g = S.seg[k];
        kk[u] = k;
        jjv[u] = j - g.off;
        limv[u] = g.bcast ? g.nfull : ((g.nfull - rank * g.s < g.s) ? g.nfull - rank * g.s : g.s);
        lov[u] = (g.part - F.grad) + jjv[u];   // local flat offset of element jj of this part
        fast[u] = live[u] && F.kind[k] != XF_METRIC && jjv[u] + 4 <= limv[u] && (lov[u] & 3) == 0;
        const long ec = fast[u] ? lov[u] : 0;
        sp[u] = *reinterpret_cast<const float4*>(A.p + ec);
        sm[u] = *reinterpret_cast<const float4*>(A.m + ec);
        sv[u] = *reinterpret_cast<const float4*>(A.v + ec);
      }
      if (i0 == 0) {
        xg_barrier(P, rank, W, 0, epoch, timeout, XG_SITE_FSDP);
        XF_STAMP(2);
      }
      float4 v[MI][W];
#pragma unroll
      for (int u = 0; u < MI; ++u) {
        const long j = base + 4 * (long)min(threadIdx.x + (i0 + u) * XG_THREADS, nv - 1);
#pragma unroll
        for (int q = 0; q < W; ++q) v[u][q] = sys_load4(rdata[q], half + rank * slice + j);
      }
#pragma unroll
      for (int u = 0; u < MI; ++u) {
        if (!live[u]) continue;
        const long j = base + 4 * (long)(threadIdx.x + (i0 + u) * XG_THREADS);
        float4 acc = v[u][0];
#pragma unroll
        for (int q = 1; q < W; ++q) acc = add4(acc, v[u][q]);
        const int k = kk[u];
        const XgSeg& g = S.seg[k];
        const long jj = jjv[u], lim = limv[u], lo = lov[u];
        const int kind = F.kind[k];
        if (kind == XF_METRIC) {
          const float* a = &acc.x;
          for (int e = 0; e < 4; ++e)
            if (jj + e < lim && jj + e < A.n_metrics) A.running[jj + e] += a[e];
          store_guard(g.part, jj, lim, z4);
          continue;
        }
        const float* ga = &acc.x;
        float pn[4] = {0.f, 0.f, 0.f, 0.f};
        if (fast[u]) {
          // writes p, m, v and the local bf16 shadow; the new p is also the published value
          const float4 pv = adam4_pre(A, lo, acc, sp[u], sm[u], sv[u], rbc1, rbc2);
          pn[0] = pv.x; pn[1] = pv.y; pn[2] = pv.z; pn[3] = pv.w;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if (jj + e >= lim) break;
            const float gr = ga[e] * A.grad_scale;
            const float mm = A.b1 * A.m[lo + e] + (1.f - A.b1) * gr;
            const float vv = A.b2 * A.v[lo + e] + (1.f - A.b2) * gr * gr;
            float pp = A.p[lo + e];
            pp -= A.lr * ((mm * rbc1) / (sqrtf(vv * rbc2) + A.eps) + A.wd * pp);
            A.m[lo + e] = mm;
            A.v[lo + e] = vv;
            A.p[lo + e] = pp;
            A.shadow[lo + e] = f2bf(pp);
            pn[e] = pp;
          }
        }
        uint2 pk;
        pk.x = (unsigned)f2bf(pn[0]) | ((unsigned)f2bf(pn[1]) << 16);
        pk.y = (unsigned)f2bf(pn[2]) | ((unsigned)f2bf(pn[3]) << 16);
        if (kind == XF_SHARD) {
          sys_store8(my_tmp, 2 * (2 * half + rank * slice + j), pk);
        } else {  // replicated: every rank holds the same update; write the full leaf directly
          bf16_t* fs = F.full_shadow[k];
          const bf16_t h4[4] = {(bf16_t)(pk.x & 0xffff), (bf16_t)(pk.x >> 16), (bf16_t)(pk.y & 0xffff),
                                (bf16_t)(pk.y >> 16)};
          for (int e = 0; e < 4; ++e)
            if (jj + e < lim) fs[jj + e] = h4[e];
        }
      }
    }
  }
  if (F.stamps) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); XF_STAMP(3); }
  xg_barrier(P, rank, W, 1, epoch, timeout, XG_SITE_FSDP);
  XF_STAMP(4);

  // phase 2: gather every peer's updated bf16 shard into the full shadow
  {
    __amdgpu_buffer_rsrc_t rtmp[W];
#pragma unroll
    for (int q = 0; q < W; ++q) rtmp[q] = sys_rsrc(P.tmp[q], bytes);
    for (int i0 = 0; i0 < nit; i0 += MI) {
      uint2 r[MI][W];
#pragma unroll
      for (int u = 0; u < MI; ++u) {
        const long j = base + 4 * (long)min(threadIdx.x + (i0 + u) * XG_THREADS, nv - 1);
#pragma unroll
        for (int q = 0; q < W; ++q) r[u][q] = sys_load8(rtmp[q], 2 * (2 * half + q * slice + j));
      }
#pragma unroll
      for (int u = 0; u < MI; ++u) {
        const int i = threadIdx.x + (i0 + u) * XG_THREADS;
        const long j = base + 4 * (long)i;
        if (i0 + u >= nit || i >= nv || j >= S.S) continue;
        const int k = xg_find(S, j);
        if (F.kind[k] != XF_SHARD) continue;
        const XgSeg& g = S.seg[k];
        const long jj = j - g.off;
#pragma unroll
        for (int q = 0; q < W; ++q) {
          const long lim = (g.nfull - q * g.s < g.s) ? g.nfull - q * g.s : g.s;
          if (jj >= lim) continue;
          bf16_t* dst = F.full_shadow[k] + seg_full_index(g, q, jj);
          if (jj + 4 <= lim) {
            *reinterpret_cast<uint2*>(dst) = r[u][q];
          } else {
            const bf16_t h4[4] = {(bf16_t)(r[u][q].x & 0xffff), (bf16_t)(r[u][q].x >> 16),
                                  (bf16_t)(r[u][q].y & 0xffff), (bf16_t)(r[u][q].y >> 16)};
            for (int e = 0; e < 4 && jj + e < lim; ++e) dst[e] = h4[e];
          }
        }
      }
    }
  }
  if (F.stamps) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); XF_STAMP(5); }
  if (threadIdx.x == 0) me->epoch[b] = epoch;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = atomicAdd(A.ticket, 1u);
    if (t == gridDim.x - 1) {
      A.step[0] = A.step[0] + 1;
      __hip_atomic_store(A.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  xg_call_done(me);
}

struct XgCtx {
  int rank = 0, world = 1;
  long cap = 0;  // floats per parity half
  float* data = nullptr;
  float* tmp = nullptr;
  XgSignal* sig = nullptr;
  XgPeers peers{};
  bool opened = false;
};

// Grid cap of every xGMI kernel (8 .. XG_MAX_BLOCKS).  With k ranks time-sharing one GPU
// (rehearsals) their spinning grids must leave every CU room for the other ranks'
// non-spinning kernels -- a peer's md_bwd that cannot be dispatched because the CUs are
// full of waiting xGMI workgroups never arrives at the barrier they wait on -- so the
// host lowers the cap (comm/xgmi.py set_max_blocks) before it creates any context; the
// layouts derived from the geometry (stage part, segment slice) follow it.
static long g_xg_max_blocks = XG_MAX_BLOCKS;
JDT_API void jdt_xgmi_set_max_blocks(int b) { g_xg_max_blocks = b < 8 ? 8 : (b > XG_MAX_BLOCKS ? XG_MAX_BLOCKS : b); }
JDT_API int jdt_xgmi_max_blocks() { return (int)g_xg_max_blocks; }

static void xg_geometry(long s, long* G_out, long* chunk_out) {
  long G = (s + 4 * XG_THREADS - 1) / (4 * XG_THREADS);
  if (G < 8) G = 8;
  if (G > g_xg_max_blocks) G = g_xg_max_blocks;
  *G_out = G;
  *chunk_out = (((s + G - 1) / G) + 3) / 4 * 4;
}

template <int OP>
static int xg_launch(XgCtx* c, const float* in, float* out, long n, long s, const XgAdam* A, long long timeout,
                     hipStream_t st, int staged = 0) {
  const int W = c->world;
  if (s <= 0 || (s & 3) || n > s * W) return -2;
  long G, chunk;
  xg_geometry(s, &G, &chunk);
  const long slice = chunk * G;
  if (slice * W > c->cap) return -3;
  if (staged && (slice != s || !A || OP != XG_ALLREDUCE)) return -2;
  XgAdam a{};
  int fuse = 0;
  if (A) { a = *A; fuse = 1; }
#define XG_CASE(w)                                                                                              \
  case w:                                                                                                       \
    hipLaunchKernelGGL((xg_kernel<w, OP>), dim3(G), dim3(XG_THREADS), 0, st, c->peers, c->rank, c->cap, in, out, \
                       n, s, slice, chunk, a, fuse, timeout, staged);                                           \
    break;
  switch (W) {
    XG_CASE(2)
    XG_CASE(3)
    XG_CASE(4)
    XG_CASE(5)
    XG_CASE(6)
    XG_CASE(7)
    XG_CASE(8)
    default:
      return -4;
  }
#undef XG_CASE
  return HIP_LAUNCH_CHECK();
}

}  // namespace jdt
using namespace jdt;

// Allocate this rank's IPC buffers (data, tmp: 2 x cap floats each; signal page)
// and export their handles (3 x 64 bytes) for the peers.
JDT_API int jdt_xgmi_create(int rank, int world, long cap_floats, void** ctx_out, void* handles_out) {
  if (world < 2 || world > XG_MAX_RANKS || rank < 0 || rank >= world) return -4;
  XgCtx* c = new XgCtx();
  c->rank = rank;
  c->world = world;
  c->cap = (cap_floats + 4 * (long)XG_MAX_BLOCKS * world + 63) / 64 * 64;
  if (2 * c->cap * (long)sizeof(float) >= 0x7fffffffL) {  // buffer-instruction offsets are 32-bit
    delete c;
    return -2;
  }
  hipIpcMemHandle_t h[3];
  // uncached: peers read these over xGMI right after the flag (see xg_barrier)
  if (ipc_alloc(reinterpret_cast<void**>(&c->data), 2 * c->cap * sizeof(float)) != hipSuccess)
    goto fail;
  if (ipc_alloc(reinterpret_cast<void**>(&c->tmp), 2 * c->cap * sizeof(float)) != hipSuccess)
    goto fail;
  if (ipc_alloc(reinterpret_cast<void**>(&c->sig), sizeof(XgSignal)) != hipSuccess)
    goto fail;
  if (hipMemset(c->sig, 0, sizeof(XgSignal)) != hipSuccess) goto fail;
  if (hipMemset(c->data, 0, 2 * c->cap * sizeof(float)) != hipSuccess) goto fail;
  if (hipMemset(c->tmp, 0, 2 * c->cap * sizeof(float)) != hipSuccess) goto fail;
  if (hipDeviceSynchronize() != hipSuccess) goto fail;
  if (hipIpcGetMemHandle(&h[0], c->data) != hipSuccess) goto fail;
  if (hipIpcGetMemHandle(&h[1], c->tmp) != hipSuccess) goto fail;
  if (hipIpcGetMemHandle(&h[2], c->sig) != hipSuccess) goto fail;
  static_assert(sizeof(hipIpcMemHandle_t) == 64, "ipc handle size");
  std::memcpy(handles_out, h, sizeof(h));
  *ctx_out = c;
  return 0;
fail:
  (void)hipGetLastError();
  ipc_release(c->data);
  ipc_release(c->tmp);
  ipc_release(c->sig);
  delete c;
  return -1;
}

// Map every peer's buffers (all_handles: world x 3 x 64 bytes, rank-major).
JDT_API int jdt_xgmi_open(void* ctx, const void* all_handles) {
  XgCtx* c = static_cast<XgCtx*>(ctx);
  const hipIpcMemHandle_t* h = static_cast<const hipIpcMemHandle_t*>(all_handles);
  for (int q = 0; q < c->world; ++q) {
    if (q == c->rank) {
      c->peers.data[q] = c->data;
      c->peers.tmp[q] = c->tmp;
      c->peers.sig[q] = c->sig;
      continue;
    }
    void* p[3] = {nullptr, nullptr, nullptr};
    for (int k = 0; k < 3; ++k) {
      if (hipIpcOpenMemHandle(&p[k], h[3 * q + k], hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
        (void)hipGetLastError();
        return -(10 + q);
      }
    }
    c->peers.data[q] = static_cast<float*>(p[0]);
    c->peers.tmp[q] = static_cast<float*>(p[1]);
    c->peers.sig[q] = static_cast<XgSignal*>(p[2]);
  }
  c->opened = true;
  return 0;
}

static long g_oneshot_bytes = -1;   // all-reduces up to this size take the one-shot kernel
static long oneshot_bytes() {
  if (g_oneshot_bytes < 0) {
    const char* e = getenv("JDT_XGMI_ONESHOT_BYTES");
    g_oneshot_bytes = e ? atol(e) : 256L * 1024;
  }
  return g_oneshot_bytes;
}
JDT_API void jdt_xgmi_set_oneshot_bytes(long b) { g_oneshot_bytes = b; }
JDT_API long jdt_xgmi_oneshot_bytes() { return oneshot_bytes(); }

static int xg_oneshot(XgCtx* c, const float* in, float* out, long n, const XgAdam* A, long long timeout,
                      hipStream_t st) {
  const long n4 = (n + 3) / 4 * 4;
  long G, chunk;
  xg_geometry(n4, &G, &chunk);
  if (G * chunk > c->cap) return -3;
  XgAdam a{};
  int fuse = 0;
  if (A) { a = *A; fuse = 1; }
#define XG_CASE(w)                                                                                              \
  case w:                                                                                                       \
    hipLaunchKernelGGL((xg_oneshot_kernel<w>), dim3(G), dim3(XG_THREADS), 0, st, c->peers, c->rank, c->cap, in, \
                       out, n, chunk, a, fuse, timeout);                                                        \
    break;
  switch (c->world) {
    XG_CASE(2)
    XG_CASE(3)
    XG_CASE(4)
    XG_CASE(5)
    XG_CASE(6)
    XG_CASE(7)
    XG_CASE(8)
    default:
      return -4;
  }
#undef XG_CASE
  return HIP_LAUNCH_CHECK();
}

JDT_API int jdt_xgmi_allreduce(void* ctx, const float* in, float* out, long n, const XgAdam* adam, long long timeout,
                               void* stream) {
  XgCtx* c = static_cast<XgCtx*>(ctx);
  if (!c->opened) return -5;
  if ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15) return -2;
  if (adam && ((adam->n_params & 3) || !adam->step || !adam->ticket)) return -2;
  if (n > 0 && n * (long)sizeof(float) <= oneshot_bytes())
    return xg_oneshot(c, in, out, n, adam, timeout, static_cast<hipStream_t>(stream));
  const long part = ((n + c->world - 1) / c->world + 3) / 4 * 4;
  return xg_launch<XG_ALLREDUCE>(c, in, out, n, part, adam, timeout, static_cast<hipStream_t>(stream));
}

// Staged all-reduce geometry: the smallest part length s >= ceil(n / world) (a
// multiple of 4) whose block split has no padding (slice == s), so that the IPC
// data buffer's layout is the flat bucket's own index; -1 if none fits.
static long xg_stage_part(int world, long n, long cap) {
  const long s0 = ((n + world - 1) / world + 3) / 4 * 4;
  for (long s = s0; s <= s0 + 16L * XG_MAX_BLOCKS; s += 4) {
    long G, chunk;
    xg_geometry(s, &G, &chunk);
    if (G * chunk == s) return s * world <= cap ? s : -1;
  }
  return -1;
}

JDT_API long jdt_xgmi_stage_part(void* ctx, long n) {
  XgCtx* c = static_cast<XgCtx*>(ctx);
  return xg_stage_part(c->world, n, c->cap);
}

// This rank's data buffer (half 0; half 1 at + capacity floats): a staged producer
// writes the bucket at base + (step & 1) * capacity, identity layout.
JDT_API float* jdt_xgmi_stage_base(void* ctx) { return static_cast<XgCtx*>(ctx)->data; }

// Zero both staging halves (positions a producer never writes -- padding between
// the bucket's views -- must reduce to zero; earlier unstaged calls leave data there).
JDT_API int jdt_xgmi_stage_clear(void* ctx, void* stream) {
  XgCtx* c = static_cast<XgCtx*>(ctx);
  return (int)hipMemsetAsync(c->data, 0, 2 * c->cap * sizeof(float), static_cast<hipStream_t>(stream));
}

// Plain (non-system-scope) global stores, exactly the store path of a staged
// producer's epilogue (mlp2_bwd / md_bwd mode 0 writing the bucket), so the
// self-test's staged steps check that path's cross-GPU visibility and not a
// copy engine's.
__global__ void __launch_bounds__(256) xg_stage_copy_kernel(float* __restrict__ dst, const float* __restrict__ src,
                                                            long n) {
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) dst[i] = src[i];
}

// Copy src[0, n) into the staging half `parity` (self-test / tools).
JDT_API int jdt_xgmi_stage_write(void* ctx, int parity, const float* src, long n, void* stream) {
  XgCtx* c = static_cast<XgCtx*>(ctx);
  if (n < 0 || n > c->cap) return -2;
  if (n == 0) return 0;
  const long g = (n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024;
  hipLaunchKernelGGL(xg_stage_copy_kernel, dim3((unsigned)g), dim3(256), 0, static_cast<hipStream_t>(stream),
                     c->data + (long)(parity & 1) * c->cap, src, n);
  return HIP_LAUNCH_CHECK();
}

// All-reduce + fused AdamW of a bucket a producer kernel already staged (see xg_kernel).
JDT_API int jdt_xgmi_allreduce_staged(void* ctx, long n, long s, const XgAdam* adam, long long timeout, void* stream) {
  XgCtx* c = static_cast<XgCtx*>(ctx);
  if (!c->opened) return -5;
  if (!adam || (adam->n_params & 3) || !adam->step || !adam->ticket) return -2;
  XgAdam a = *adam;
  a.zero = nullptr;  // the producer overwrites every bucket element it owns each step
  return xg_launch<XG_ALLREDUCE>(c, nullptr, nullptr, n, s, &a, timeout, static_cast<hipStream_t>(stream), 1);
}

// Part length s (multiple of 4, n <= world*s): out[0, s) receives the sum of
// elements [rank*s, rank*s + s) (valid up to n).
JDT_API int jdt_xgmi_reduce_scatter(void* ctx, const float* in, float* out, long n, long s, long long timeout,
                                    void* stream) {
  XgCtx* c = static_cast<XgCtx*>(ctx);
  if (!c->opened) return -5;
  if ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15) return -2;
  return xg_launch<XG_REDUCE_SCATTER>(c, in, out, n, s, nullptr, timeout, static_cast<hipStream_t>(stream));
}

// in[0, s) of every rank -> out[q*s + j] (valid up to n).
JDT_API int jdt_xgmi_all_gather(void* ctx, const float* in, float* out, long n, long s, long long timeout,
                                void* stream) {
  XgCtx* c = static_cast<XgCtx*>(ctx);
  if (!c->opened) return -5;
  if ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15) return -2;
  return xg_launch<XG_ALL_GATHER>(c, in, out, n, s, nullptr, timeout, static_cast<hipStream_t>(stream));
}

// Segmented RS (op 1) / AG (op 2) over up to 16 tensors; see XgSegs.
JDT_API int jdt_xgmi_segments(void* ctx, const XgSegs* segs, int op, int accumulate, long long timeout,
                              void* stream) {
  XgCtx* c = static_cast<XgCtx*>(ctx);
  if (!c->opened) return -5;
  if (segs->n < 1 || segs->n > XG_MAX_SEGS) return -2;
  long off = 0;
  for (int k = 0; k < segs->n; ++k) {
    const XgSeg& g = segs->seg[k];
    if ((g.s & 3) || g.off != off || g.nfull > g.s * c->world) return -2;
    if (g.bcast && (op != XG_REDUCE_SCATTER || g.nfull > g.s || g.rows > 1)) return -2;
    if (g.rows > 1) {
      const long w = g.s / g.rows;
      if (g.s % g.rows || (w & 3) || (g.ld & 3) || (g.qoff & 3) || g.qoff < w ||
          (long)(c->world - 1) * g.qoff + w > g.ld || g.rows * g.ld > g.nfull)
        return -2;
    }
    if ((reinterpret_cast<uintptr_t>(g.full) | reinterpret_cast<uintptr_t>(g.part)) & 15) return -2;
    off += g.s;
  }
  if (off != segs->S || off <= 0) return -2;
  long G, chunk;
  xg_geometry(off, &G, &chunk);
  const long slice = chunk * G;
  if (slice * c->world > c->cap) return -3;
  hipStream_t st = static_cast<hipStream_t>(stream);
#define XG_SEG_CASE(w)                                                                                         \
  case w:                                                                                                      \
    if (op == XG_REDUCE_SCATTER)                                                                               \
      hipLaunchKernelGGL((xg_seg_kernel<w, XG_REDUCE_SCATTER>), dim3(G), dim3(XG_THREADS), 0, st, c->peers,    \
                         c->rank, c->cap, *segs, slice, chunk, accumulate, timeout);                          \
    else                                                                                                       \
      hipLaunchKernelGGL((xg_seg_kernel<w, XG_ALL_GATHER>), dim3(G), dim3(XG_THREADS), 0, st, c->peers,        \
                         c->rank, c->cap, *segs, slice, chunk, accumulate, timeout);                          \
    break;
  if (op != XG_REDUCE_SCATTER && op != XG_ALL_GATHER) return -2;
  switch (c->world) {
    XG_SEG_CASE(2)
    XG_SEG_CASE(3)
    XG_SEG_CASE(4)
    XG_SEG_CASE(5)
    XG_SEG_CASE(6)
    XG_SEG_CASE(7)
    XG_SEG_CASE(8)
    default:
      return -4;
  }
#undef XG_SEG_CASE
  return HIP_LAUNCH_CHECK();
}

JDT_API int jdt_xgmi_segs_size() { return (int)sizeof(XgSegs); }
JDT_API int jdt_xgmi_fsdp_size() { return (int)sizeof(XgFsdp); }

// One FSDP step's communication + sharded AdamW + metrics fold (xg_fsdp_kernel).
// Segment word sizes: fp32 grads; the bf16 full shadows get the same element index.
JDT_API int jdt_xgmi_fsdp_step(void* ctx, const XgSegs* segs, const XgFsdp* f, long long timeout, void* stream) {
  XgCtx* c = static_cast<XgCtx*>(ctx);
  if (!c->opened) return -5;
  if (segs->n < 1 || segs->n > XG_MAX_SEGS || !f->A.step || !f->A.ticket || !f->A.p || !f->A.m || !f->A.v ||
      !f->A.shadow || !f->grad)
    return -2;
  long off = 0;
  for (int k = 0; k < segs->n; ++k) {
    const XgSeg& g = segs->seg[k];
    if ((g.s & 3) || g.off != off || g.nfull > g.s * c->world) return -2;
    if (g.bcast && (g.nfull > g.s || g.rows > 1)) return -2;
    if ((f->kind[k] == XF_SHARD) == (g.bcast != 0)) return -2;          // sharded <=> not all-reduce
    if (f->kind[k] != XF_METRIC && !f->full_shadow[k]) return -2;
    if (f->kind[k] == XF_METRIC && g.part != g.full) return -2;
    if (g.rows > 1) {
      const long w = g.s / g.rows;
      if (g.s % g.rows || (w & 3) || (g.ld & 3) || (g.qoff & 3) || g.qoff < w ||
          (long)(c->world - 1) * g.qoff + w > g.ld || g.rows * g.ld > g.nfull)
        return -2;
    }
    if ((reinterpret_cast<uintptr_t>(g.full) | reinterpret_cast<uintptr_t>(g.part)) & 15) return -2;
    if (f->full_shadow[k] && (reinterpret_cast<uintptr_t>(f->full_shadow[k]) & 7)) return -2;
    off += g.s;
  }
  if (off != segs->S || off <= 0) return -2;
  long G, chunk;
  xg_geometry(off, &G, &chunk);
  const long slice = chunk * G;
  if (slice * c->world > c->cap) return -3;
  hipStream_t st = static_cast<hipStream_t>(stream);
#define XG_F_CASE(w)                                                                                          \
  case w:                                                                                                     \
    hipLaunchKernelGGL((xg_fsdp_kernel<w>), dim3(G), dim3(XG_THREADS), 0, st, c->peers, c->rank, c->cap, *segs, \
                       *f, slice, chunk, timeout);                                                           \
    break;
  switch (c->world) {
    XG_F_CASE(2)
    XG_F_CASE(3)
    XG_F_CASE(4)
    XG_F_CASE(5)
    XG_F_CASE(6)
    XG_F_CASE(7)
    XG_F_CASE(8)
    default:
      return -4;
  }
#undef XG_F_CASE
  return HIP_LAUNCH_CHECK();
}

JDT_API int jdt_xgmi_adam_size() { return (int)sizeof(XgAdam); }
JDT_API int jdt_stage_map_size() { return (int)sizeof(StageMap); }

// Per-peer slot stride (floats) of a segmented / fused FSDP launch over S packed words.
JDT_API long jdt_xgmi_seg_slice(long S) {
  long G, chunk;
  xg_geometry(S, &G, &chunk);
  return G * chunk;
}

JDT_API long jdt_xgmi_capacity(void* ctx) { return static_cast<XgCtx*>(ctx)->cap; }

// The first timeout's [site, block, epoch, peer] (zeros if none; synchronises the device).
JDT_API int jdt_xgmi_error_info(void* ctx, unsigned* out4) {
  XgCtx* c = static_cast<XgCtx*>(ctx);
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpy(out4, c->sig->errinfo, 4 * sizeof(unsigned), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return 0;
}

// 1 if any barrier of this rank timed out (synchronises the device).
JDT_API int jdt_xgmi_error(void* ctx) {
  XgCtx* c = static_cast<XgCtx*>(ctx);
  int e = 0;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpy(&e, &c->sig->err, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return e;
}

// Teardown phase 1 (collective with phase 2 through a barrier, comm/xgmi.py close): drain
// this rank's queue and close its mappings of the peers' buffers.  Only after EVERY rank
// did so does any rank release its own exported buffers (jdt_xgmi_destroy), so no peer
// mapping outlives the pages it resolves to.
JDT_API int jdt_xgmi_unmap(void* ctx) {
  XgCtx* c = static_cast<XgCtx*>(ctx);
  if (!c) return 0;
  (void)hipDeviceSynchronize();
  if (c->opened) {
    for (int q = 0; q < c->world; ++q) {
      if (q == c->rank) continue;
      if (c->peers.data[q]) (void)hipIpcCloseMemHandle(c->peers.data[q]);
      if (c->peers.tmp[q]) (void)hipIpcCloseMemHandle(c->peers.tmp[q]);
      if (c->peers.sig[q]) (void)hipIpcCloseMemHandle(c->peers.sig[q]);
      c->peers.data[q] = c->peers.tmp[q] = nullptr;
      c->peers.sig[q] = nullptr;
    }
    c->opened = false;
  }
  return 0;
}

JDT_API int jdt_xgmi_destroy(void* ctx) {
  XgCtx* c = static_cast<XgCtx*>(ctx);
  if (!c) return 0;
  (void)jdt_xgmi_unmap(ctx);   // one-phase fallback (garbage collection): unmap, then release
  ipc_release(c->data);
  ipc_release(c->tmp);
  ipc_release(c->sig);
  delete c;
  return 0;
}
