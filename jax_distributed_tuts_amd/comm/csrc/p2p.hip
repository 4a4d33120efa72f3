// Stage-to-stage activation hand-off for pipeline parallelism over xGMI
// (the GPipe ppermute between neighbouring stages).
//
// RCCL send/recv costs tens of microseconds per call and cannot be replayed
// inside a per-rank hipGraph without the peer's graph being in lock-step, while
// a GPipe tick of the tutorial MLP is a handful of microseconds of compute.
// Here every rank owns an IPC-exported *inbox*: n_slots fixed-size slots in
// uncached device memory plus a signal page.  A send is a kernel on the
// producer that pushes the tensor straight into the consumer's inbox slot over
// the xGMI link (posted remote stores, no round trip) and then raises one epoch
// flag per block (relaxed system-scope store after the data stores are
// acknowledged; payload stores and loads are system-scope sc0 sc1 buffer
// instructions, common.h, so no cache maintenance); a receive is a kernel on the
// consumer that waits for the flags of its own blocks and copies the slot into
// a local tensor.  Both are ordinary kernels on the caller's stream, so a whole
// pipeline step -- compute, sends and receives -- is one hipGraph per rank.
//
// Epochs: the flag value is (*epoch_src + 1), where epoch_src is the device
// step counter of the optimizer (read before it is advanced at the end of the
// step), so graph replays need no host-side bookkeeping.  Every stage advances
// its own counter once per step, in lock-step with its neighbours.
//
// Slot reuse without a back-channel: in a GPipe step the producer writes slot i
// of step k+1 only after it has received every activation gradient of step k,
// and the consumer sends those gradients only after the kernels that read slot i
// of step k have completed (stream order) -- so one buffer per (direction,
// microbatch) is race-free.  The consumer's sc0 sc1 loads see the peer's
// write-through stores once the flag is observed, on every XCD.
//
// Waits time out (s_memrealtime, 100 MHz) into an error flag, never a hang.
#include "common.h"
#include "ipc_pool.h"

#include <cstddef>
#include <cstring>

namespace jdt {

constexpr int P2P_MAX_RANKS = 8;
constexpr int P2P_MAX_SLOTS = 64;
constexpr int P2P_MAX_BLOCKS = 32;
constexpr int P2P_THREADS = 256;
constexpr long P2P_BLOCK_BYTES = 8192;  // bytes per block per call (>= 2 uint4 per thread)

struct P2PSignal {
  unsigned flag[P2P_MAX_SLOTS][P2P_MAX_BLOCKS];
  int err;
};

struct P2PPeers {
  char* inbox[P2P_MAX_RANKS];
  P2PSignal* sig[P2P_MAX_RANKS];
};

struct P2PCtx {
  int rank = 0, world = 1;
  long slot_bytes = 0;
  int n_slots = 0;
  char* inbox = nullptr;
  P2PSignal* sig = nullptr;
  P2PPeers peers{};
  bool opened = false;
};

__device__ __forceinline__ unsigned long long p2p_now() { return __builtin_amdgcn_s_memrealtime(); }

static inline int p2p_blocks(long nbytes) {
  long g = (nbytes + P2P_BLOCK_BYTES - 1) / P2P_BLOCK_BYTES;
  if (g < 1) g = 1;
  if (g > P2P_MAX_BLOCKS) g = P2P_MAX_BLOCKS;
  return (int)g;
}

// Block b moves 16-byte words [b*per, min((b+1)*per, nw)).
__device__ __forceinline__ void p2p_range(long nw, long* lo, long* hi) {
  const long per = (nw + gridDim.x - 1) / gridDim.x;
  *lo = (long)blockIdx.x * per;
  *hi = *lo + per < nw ? *lo + per : nw;
}

__global__ void __launch_bounds__(P2P_THREADS) p2p_send_kernel(const uint4* __restrict__ src, uint4* dst, long nw,
                                                               unsigned* flag, const int* epoch_src) {
  long lo, hi;
  p2p_range(nw, &lo, &hi);
  // remote stores into the peer's inbox: system-scope write-through (sc0 sc1, common.h)
  const __amdgpu_buffer_rsrc_t rd = sys_rsrc(dst, (unsigned long long)nw * 16ull);
  for (long i = lo + threadIdx.x; i < hi; i += P2P_THREADS)
    sys_store4(rd, 4 * i, __builtin_bit_cast(float4, src[i]));
  // every storing wave drains its write-through stores before the barrier that
  // precedes the flag (no release fence: that would write back the whole L2 per wave)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned epoch = (unsigned)epoch_src[0] + 1u;
    __hip_atomic_store(&flag[blockIdx.x], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ void __launch_bounds__(P2P_THREADS) p2p_recv_kernel(const uint4* src, uint4* __restrict__ dst, long nw,
                                                               unsigned* flag, const int* epoch_src, int* err,
                                                               long long timeout) {
  if (threadIdx.x == 0) {
    const unsigned epoch = (unsigned)epoch_src[0] + 1u;
    const unsigned long long t0 = p2p_now();
    while ((int)(__hip_atomic_load(&flag[blockIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
      if ((long long)(p2p_now() - t0) > timeout) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  long lo, hi;
  p2p_range(nw, &lo, &hi);
  // every load of the handed-off bytes is a system-scope sc0 sc1 load (common.h)
  const __amdgpu_buffer_rsrc_t rs = sys_rsrc(src, (unsigned long long)nw * 16ull);
  for (long i = lo + threadIdx.x; i < hi; i += P2P_THREADS) dst[i] = __builtin_bit_cast(uint4, sys_load4(rs, 4 * i));
}

}  // namespace jdt
using namespace jdt;

// Allocate this rank's inbox (n_slots x slot_bytes, uncached) and signal page;
// export their IPC handles (2 x 64 bytes).
JDT_API int jdt_p2p_create(int rank, int world, long slot_bytes, int n_slots, void** ctx_out, void* handles_out) {
  if (world < 2 || world > P2P_MAX_RANKS || rank < 0 || rank >= world) return -4;
  if (n_slots < 1 || n_slots > P2P_MAX_SLOTS || slot_bytes <= 0) return -2;
  P2PCtx* c = new P2PCtx();
  c->rank = rank;
  c->world = world;
  c->slot_bytes = (slot_bytes + 255) / 256 * 256;
  c->n_slots = n_slots;
  hipIpcMemHandle_t h[2];
  const size_t inbox_bytes = (size_t)c->slot_bytes * n_slots;
  if (ipc_alloc(reinterpret_cast<void**>(&c->inbox), inbox_bytes) != hipSuccess)
    goto fail;
  if (ipc_alloc(reinterpret_cast<void**>(&c->sig), sizeof(P2PSignal)) != hipSuccess)
    goto fail;
  if (hipMemset(c->inbox, 0, inbox_bytes) != hipSuccess) goto fail;
  if (hipMemset(c->sig, 0, sizeof(P2PSignal)) != hipSuccess) goto fail;
  if (hipDeviceSynchronize() != hipSuccess) goto fail;
  if (hipIpcGetMemHandle(&h[0], c->inbox) != hipSuccess) goto fail;
  if (hipIpcGetMemHandle(&h[1], c->sig) != hipSuccess) goto fail;
  std::memcpy(handles_out, h, sizeof(h));
  *ctx_out = c;
  return 0;
fail:
  (void)hipGetLastError();
  ipc_release(c->inbox);
  ipc_release(c->sig);
  delete c;
  return -1;
}

// Map every peer's inbox + signal page (all_handles: world x 2 x 64 bytes).
JDT_API int jdt_p2p_open(void* ctx, const void* all_handles) {
  P2PCtx* c = static_cast<P2PCtx*>(ctx);
  const hipIpcMemHandle_t* h = static_cast<const hipIpcMemHandle_t*>(all_handles);
  for (int q = 0; q < c->world; ++q) {
    if (q == c->rank) {
      c->peers.inbox[q] = c->inbox;
      c->peers.sig[q] = c->sig;
      continue;
    }
    void* p[2] = {nullptr, nullptr};
    for (int k = 0; k < 2; ++k) {
      if (hipIpcOpenMemHandle(&p[k], h[2 * q + k], hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
        (void)hipGetLastError();
        return -(10 + q);
      }
    }
    c->peers.inbox[q] = static_cast<char*>(p[0]);
    c->peers.sig[q] = static_cast<P2PSignal*>(p[1]);
  }
  c->opened = true;
  return 0;
}

static int p2p_check(P2PCtx* c, int slot, const void* a, long nbytes) {
  if (!c || !c->opened) return -5;
  if (slot < 0 || slot >= c->n_slots) return -2;
  if (nbytes <= 0 || nbytes > c->slot_bytes || (nbytes & 15)) return -2;
  if (reinterpret_cast<uintptr_t>(a) & 15) return -2;
  return 0;
}

// Push src[0, nbytes) into peer `to`'s inbox slot; flag = *epoch_src + 1.
JDT_API int jdt_p2p_send(void* ctx, int to, int slot, const void* src, long nbytes, const int* epoch_src,
                         void* stream) {
  P2PCtx* c = static_cast<P2PCtx*>(ctx);
  if (int rc = p2p_check(c, slot, src, nbytes)) return rc;
  if (to < 0 || to >= c->world || to == c->rank) return -2;
  const int G = p2p_blocks(nbytes);
  uint4* dst = reinterpret_cast<uint4*>(c->peers.inbox[to] + (size_t)slot * c->slot_bytes);
  unsigned* flag = c->peers.sig[to]->flag[slot];
  hipLaunchKernelGGL(p2p_send_kernel, dim3(G), dim3(P2P_THREADS), 0, static_cast<hipStream_t>(stream),
                     static_cast<const uint4*>(src), dst, nbytes / 16, flag, epoch_src);
  return HIP_LAUNCH_CHECK();
}

// Wait for this rank's inbox slot (flag >= *epoch_src + 1) and copy it to dst.
// nbytes must equal the sender's (same block split).
JDT_API int jdt_p2p_recv(void* ctx, int slot, void* dst, long nbytes, const int* epoch_src, long long timeout,
                         void* stream) {
  P2PCtx* c = static_cast<P2PCtx*>(ctx);
  if (int rc = p2p_check(c, slot, dst, nbytes)) return rc;
  const int G = p2p_blocks(nbytes);
  const uint4* src = reinterpret_cast<const uint4*>(c->inbox + (size_t)slot * c->slot_bytes);
  hipLaunchKernelGGL(p2p_recv_kernel, dim3(G), dim3(P2P_THREADS), 0, static_cast<hipStream_t>(stream), src,
                     static_cast<uint4*>(dst), nbytes / 16, c->sig->flag[slot], epoch_src, &c->sig->err, timeout);
  return HIP_LAUNCH_CHECK();
}

JDT_API long jdt_p2p_slot_bytes(void* ctx) { return static_cast<P2PCtx*>(ctx)->slot_bytes; }

// 1 if any receive of this rank timed out (synchronises the device).
JDT_API int jdt_p2p_error(void* ctx) {
  P2PCtx* c = static_cast<P2PCtx*>(ctx);
  int e = 0;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpy(&e, &c->sig->err, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  return e;
}

// Zero this rank's flags and error word (after the start-up self-test).
JDT_API int jdt_p2p_reset(void* ctx) {
  P2PCtx* c = static_cast<P2PCtx*>(ctx);
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemset(c->sig, 0, sizeof(P2PSignal)) != hipSuccess) return -1;
  return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

// Teardown phase 1 (see jdt_xgmi_unmap): close this rank's mappings of its peers' pages.
JDT_API int jdt_p2p_unmap(void* ctx) {
  P2PCtx* c = static_cast<P2PCtx*>(ctx);
  if (!c) return 0;
  (void)hipDeviceSynchronize();
  if (c->opened) {
    for (int q = 0; q < c->world; ++q) {
      if (q == c->rank) continue;
      if (c->peers.inbox[q]) (void)hipIpcCloseMemHandle(c->peers.inbox[q]);
      if (c->peers.sig[q]) (void)hipIpcCloseMemHandle(c->peers.sig[q]);
      c->peers.inbox[q] = nullptr;
      c->peers.sig[q] = nullptr;
    }
    c->opened = false;
  }
  return 0;
}

JDT_API int jdt_p2p_destroy(void* ctx) {
  P2PCtx* c = static_cast<P2PCtx*>(ctx);
  if (!c) return 0;
  (void)jdt_p2p_unmap(ctx);
  ipc_release(c->inbox);
  ipc_release(c->sig);
  delete c;
  return 0;
}

// Raw view of rank q's inbox and signal page for kernels that hand off in-kernel
// (ops/csrc/pp_stage.hip): inbox base, flag array [P2P_MAX_SLOTS][P2P_MAX_BLOCKS] and
// error word of q's page (q = this rank: its own).  -2 if q is out of range or unmapped.
JDT_API int jdt_p2p_peer(void* ctx, int q, void** inbox, void** flags, void** err) {
  P2PCtx* c = static_cast<P2PCtx*>(ctx);
  if (!c || !c->opened || q < 0 || q >= c->world) return -2;
  // addresses only (device pointers, nothing is dereferenced on the host)
  char* sig = reinterpret_cast<char*>(c->peers.sig[q]);
  *inbox = c->peers.inbox[q];
  *flags = sig + offsetof(P2PSignal, flag);
  *err = sig + offsetof(P2PSignal, err);
  return 0;
}
JDT_API int jdt_p2p_max_blocks() { return P2P_MAX_BLOCKS; }
JDT_API int jdt_p2p_max_slots() { return P2P_MAX_SLOTS; }
