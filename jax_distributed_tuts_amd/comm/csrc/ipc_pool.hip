// Pool of IPC-exported buffers (ipc_pool.h).
//
// Why: bench.py's autotune builds and tears down a dozen trainers per process, each with
// its own xGMI / p2p / tile-exchange context.  With the buffers returned to the driver
// at every teardown, a context's start-up self-test on 4 ranks sharing one GPU failed
// about once in four runs (profiles/r5_ipc_pool.txt): after torch.cuda.synchronize the
// rank's OWN freshly computed tensors kept changing -- foreign writes into pages this
// process had just re-allocated.  Teardown was collective (runtime.dist.quiesce: no
// kernel of any rank in flight), but each rank closed its peer mappings and freed its own
// buffers in ONE call, so a rank could free (and re-allocate into torch) pages a slower
// peer still had mapped.  Teardown is now two-phase (every rank closes its mappings of
// the peers' pages, a barrier, then every rank releases its own: jdt_*_unmap, then
// jdt_*_destroy), and the pool is an option on top (JDT_IPC_POOL, default on): a
// released buffer is kept for the next context of the same size instead of going back to
// the driver.  JDT_IPC_POOL=0 frees at release (tools/xgmi_churn.py measures both); the
// pool frees instead of keeping once it holds more than JDT_IPC_POOL_MB (default 512).
#include "common.h"
#include "ipc_pool.h"

#include <cstdlib>
#include <mutex>
#include <vector>

namespace jdt {
namespace {

struct PoolBuf {
  void* p;
  size_t bytes;
  int dev;
  bool used;
};

std::mutex g_pool_mu;
std::vector<PoolBuf> g_pool;

bool pool_on() {
  static const bool on = [] {
    const char* e = getenv("JDT_IPC_POOL");
    return !(e && e[0] == '0');
  }();
  return on;
}
size_t pool_cap_bytes() {
  static const size_t cap = [] {
    const char* e = getenv("JDT_IPC_POOL_MB");
    const long mb = e ? atol(e) : 512;
    return (size_t)(mb > 0 ? mb : 0) << 20;
  }();
  return cap;
}

}  // namespace

hipError_t ipc_alloc(void** out, size_t bytes) {
  *out = nullptr;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> lk(g_pool_mu);
  if (pool_on()) {
    for (auto& b : g_pool) {
      if (!b.used && b.bytes == bytes && b.dev == dev) {
        b.used = true;
        *out = b.p;
        return hipSuccess;
      }
    }
  }
  void* p = nullptr;
  e = hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return e;
  g_pool.push_back({p, bytes, dev, true});
  *out = p;
  return hipSuccess;
}

void ipc_release(void* p) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(g_pool_mu);
  size_t kept = 0;
  for (const auto& b : g_pool)
    if (!b.used) kept += b.bytes;
  for (size_t i = 0; i < g_pool.size(); ++i) {
    if (g_pool[i].p != p) continue;
    if (pool_on() && kept + g_pool[i].bytes <= pool_cap_bytes()) {
      g_pool[i].used = false;
    } else {
      // pool off or full: back to the driver (safe: teardown is two-phase, every peer has
      // closed its mapping of these pages before any rank releases them)
      (void)hipFree(g_pool[i].p);
      g_pool.erase(g_pool.begin() + (long)i);
    }
    return;
  }
}

}  // namespace jdt

// Pool census: out[0] buffers, out[1] bytes, out[2] buffers in use.
JDT_API void jdt_ipc_pool_stats(long* out) {
  std::lock_guard<std::mutex> lk(jdt::g_pool_mu);
  long n = 0, bytes = 0, used = 0;
  for (const auto& b : jdt::g_pool) {
    ++n;
    bytes += (long)b.bytes;
    used += b.used ? 1 : 0;
  }
  out[0] = n;
  out[1] = bytes;
  out[2] = used;
}
