// IPC buffers of the per-tile gradient exchange that lets the fused 2-layer DP step run
// as ONE launch per step at N > 1 (ops/csrc/common.h TxArgs; the exchange itself is in
// ops/csrc/mlp_fused.hip, mlp2_bwd AHEAD with Mlp2Args::tx).
//
// Per rank: a partial inbox [tiles][TX_MAX_RANKS][pay] floats (peer src pushes its
// partial tile T into slot [T][src] of T's owner), a reduced inbox [tiles][pay] floats
// (the owner pushes the summed tile into every peer's slot [T]) and a signal page of
// epoch flags.  All three are uncached device memory: peers write them over xGMI with
// system-scope write-through stores and this GPU reads them with system-scope loads
// right after a flag (the same discipline as comm/csrc/xgmi.hip and p2p.hip).  The
// TxArgs the kernel reads (every rank's mapped pointers) lives in device memory.
#include "common.h"
#include "ipc_pool.h"

#include <cstring>

namespace jdt {

struct TxCtx {
  int rank = 0, world = 1, tiles = 0, pay = 0;
  float* part = nullptr;
  float* red = nullptr;
  unsigned* flag = nullptr;
  unsigned* err = nullptr;   // local error word (TxArgs::err)
  TxArgs host{};
  TxArgs* dev = nullptr;   // device copy of `host`
  bool opened = false;
};

static long tx_part_floats(const TxCtx* c) { return (long)c->tiles * TX_MAX_RANKS * c->pay; }
static long tx_red_floats(const TxCtx* c) { return (long)c->tiles * c->pay; }
// [tile][src] partial flags, [tile] reduced flags (DP), [tile][owner] updated-value flags (FSDP)
static long tx_flag_words(const TxCtx* c) { return (long)c->tiles * TX_MAX_RANKS * 2 + c->tiles; }

}  // namespace jdt
using namespace jdt;

// Allocate this rank's inboxes and signal page, export their IPC handles (3 x 64 bytes).
JDT_API int jdt_tx_create(int rank, int world, int tiles, int pay, void** ctx_out, void* handles_out) {
  if (world < 2 || world > TX_MAX_RANKS || rank < 0 || rank >= world) return -4;
  if (tiles <= 0 || pay <= 0 || pay % 4) return -2;
  TxCtx* c = new TxCtx();
  c->rank = rank;
  c->world = world;
  c->tiles = tiles;
  c->pay = pay;
  hipIpcMemHandle_t h[3];
  if ((long)tx_part_floats(c) * (long)sizeof(float) >= 0x7fffffffL) goto fail;   // 32-bit buffer offsets
  if (ipc_alloc(reinterpret_cast<void**>(&c->part), tx_part_floats(c) * sizeof(float)) != hipSuccess)
    goto fail;
  if (ipc_alloc(reinterpret_cast<void**>(&c->red), tx_red_floats(c) * sizeof(float)) != hipSuccess)
    goto fail;
  if (ipc_alloc(reinterpret_cast<void**>(&c->flag), tx_flag_words(c) * sizeof(unsigned)) != hipSuccess)
    goto fail;
  if (hipMemset(c->part, 0, tx_part_floats(c) * sizeof(float)) != hipSuccess) goto fail;
  if (hipMemset(c->red, 0, tx_red_floats(c) * sizeof(float)) != hipSuccess) goto fail;
  if (hipMemset(c->flag, 0, tx_flag_words(c) * sizeof(unsigned)) != hipSuccess) goto fail;
  if (hipMalloc(reinterpret_cast<void**>(&c->dev), sizeof(TxArgs)) != hipSuccess) goto fail;
  if (hipMalloc(reinterpret_cast<void**>(&c->err), sizeof(unsigned)) != hipSuccess) goto fail;
  if (hipMemset(c->err, 0, sizeof(unsigned)) != hipSuccess) goto fail;
  if (hipDeviceSynchronize() != hipSuccess) goto fail;
  if (hipIpcGetMemHandle(&h[0], c->part) != hipSuccess) goto fail;
  if (hipIpcGetMemHandle(&h[1], c->red) != hipSuccess) goto fail;
  if (hipIpcGetMemHandle(&h[2], c->flag) != hipSuccess) goto fail;
  static_assert(sizeof(hipIpcMemHandle_t) == 64, "ipc handle size");
  std::memcpy(handles_out, h, sizeof(h));
  *ctx_out = c;
  return 0;
fail:
  (void)hipGetLastError();
  ipc_release(c->part);
  ipc_release(c->red);
  ipc_release(c->flag);
  if (c->dev) (void)hipFree(c->dev);
  if (c->err) (void)hipFree(c->err);
  delete c;
  return -1;
}

// Map every peer's buffers (all_handles: world x 3 x 64 bytes, rank-major) and upload
// the kernel's TxArgs.
JDT_API int jdt_tx_open(void* ctx, const void* all_handles, long long timeout_ticks) {
  TxCtx* c = static_cast<TxCtx*>(ctx);
  const hipIpcMemHandle_t* h = static_cast<const hipIpcMemHandle_t*>(all_handles);
  TxArgs& A = c->host;
  std::memset(&A, 0, sizeof(A));
  for (int q = 0; q < c->world; ++q) {
    if (q == c->rank) {
      A.part[q] = c->part;
      A.red[q] = c->red;
      A.flag[q] = c->flag;
      continue;
    }
    void* p = nullptr;
    if (hipIpcOpenMemHandle(&p, h[3 * q + 0], hipIpcMemLazyEnablePeerAccess) != hipSuccess) return -1;
    A.part[q] = static_cast<float*>(p);
    if (hipIpcOpenMemHandle(&p, h[3 * q + 1], hipIpcMemLazyEnablePeerAccess) != hipSuccess) return -1;
    A.red[q] = static_cast<float*>(p);
    if (hipIpcOpenMemHandle(&p, h[3 * q + 2], hipIpcMemLazyEnablePeerAccess) != hipSuccess) return -1;
    A.flag[q] = static_cast<unsigned*>(p);
  }
  A.rank = c->rank;
  A.world = c->world;
  A.tiles = c->tiles;
  A.pay = c->pay;
  A.timeout = timeout_ticks;
  A.err = c->err;
  if (hipMemcpy(c->dev, &A, sizeof(A), hipMemcpyHostToDevice) != hipSuccess) return -1;
  c->opened = true;
  return 0;
}

// Device pointer of the TxArgs (Mlp2Args::tx), or null before jdt_tx_open.
JDT_API void* jdt_tx_args(void* ctx) {
  TxCtx* c = static_cast<TxCtx*>(ctx);
  return c->opened ? c->dev : nullptr;
}

JDT_API int jdt_tx_args_size() { return (int)sizeof(TxArgs); }

// Zero this rank's flags (after the self-test, before any step kernel: the step kernels'
// epochs start at 1).  Every rank resets its own page, then the ranks meet at a barrier.
JDT_API int jdt_tx_reset(void* ctx) {
  TxCtx* c = static_cast<TxCtx*>(ctx);
  if (hipMemset(c->flag, 0, tx_flag_words(c) * sizeof(unsigned)) != hipSuccess) return -1;
  return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

// Teardown phase 1 (see jdt_xgmi_unmap): close this rank's mappings of its peers' pages.
JDT_API void jdt_tx_unmap(void* ctx) {
  TxCtx* c = static_cast<TxCtx*>(ctx);
  if (!c) return;
  (void)hipDeviceSynchronize();
  for (int q = 0; q < c->world && c->opened; ++q) {
    if (q == c->rank) continue;
    if (c->host.part[q]) (void)hipIpcCloseMemHandle(c->host.part[q]);
    if (c->host.red[q]) (void)hipIpcCloseMemHandle(c->host.red[q]);
    if (c->host.flag[q]) (void)hipIpcCloseMemHandle(c->host.flag[q]);
    c->host.part[q] = c->host.red[q] = nullptr;
    c->host.flag[q] = nullptr;
  }
  c->opened = false;
}

JDT_API void jdt_tx_close(void* ctx) {
  TxCtx* c = static_cast<TxCtx*>(ctx);
  if (!c) return;
  jdt_tx_unmap(ctx);
  ipc_release(c->part);
  ipc_release(c->red);
  ipc_release(c->flag);
  if (c->dev) (void)hipFree(c->dev);
  if (c->err) (void)hipFree(c->err);
  delete c;
}

// The error word (bit 2: an exchange wait timed out), read synchronously.
JDT_API unsigned jdt_tx_error(void* ctx) {
  TxCtx* c = static_cast<TxCtx*>(ctx);
  unsigned v = 0;
  if (!c || !c->err || hipMemcpy(&v, c->err, sizeof(v), hipMemcpyDeviceToHost) != hipSuccess) return 0xffffffffu;
  return v;
}
