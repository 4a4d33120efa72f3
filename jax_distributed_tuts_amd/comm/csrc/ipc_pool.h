// Process-wide pool of the uncached device buffers the comm contexts export over IPC
// (xgmi.hip, p2p.hip, tile_exchange.hip).  A released buffer goes back to the pool, not
// to the driver, and the next context asking for the same size on the same device gets
// it again: IPC-exported pages are never recycled into this process's other allocations
// while a peer process may still hold a mapping of them.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

namespace jdt {

// An uncached (hipDeviceMallocUncached) buffer of exactly `bytes` on the current device:
// a released pooled one of that size, else a new allocation.  Contents are undefined.
hipError_t ipc_alloc(void** p, size_t bytes);
// Return a buffer from ipc_alloc to the pool (null: no-op).
void ipc_release(void* p);

}  // namespace jdt
