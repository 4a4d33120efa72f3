// Pool of IPC-exported buffers (ipc_pool.h).
//
// Why: bench.py's autotune builds and tears down a dozen trainers per process, each with
// its own xGMI / p2p / tile-exchange context.  With the buffers returned to the driver
// at every teardown, a context's start-up self-test on 4 ranks sharing one GPU failed
// about once in four runs (profiles/r5_ipc_pool.txt): after torch.cuda.synchronize the
// rank's OWN freshly computed tensors kept changing -- foreign writes into pages this
// process had just re-allocated.  Teardown was already collective (runtime.dist.quiesce:
// no kernel of any rank in flight), so the writes came through a peer's mapping that
// still resolved to the freed pages.  Keeping exported pages for the life of the process
// removes the recycling; the pool is small (a few MB per context size).
#include "common.h"
#include "ipc_pool.h"

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

}  // namespace

hipError_t ipc_alloc(void** out, size_t bytes) {
  *out = nullptr;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> lk(g_pool_mu);
  for (auto& b : g_pool) {
    if (!b.used && b.bytes == bytes && b.dev == dev) {
      b.used = true;
      *out = b.p;
      return hipSuccess;
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
  for (auto& b : g_pool) {
    if (b.p == p) {
      b.used = false;
      return;
    }
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
