// Grid-barrier micro-benchmark (tools/barrier_lab.py): what a persistent multi-step
// launch of the headline step would pay per step in place of the kernel boundary.
//
//   kind 0 (flat):  every workgroup adds 1 to ONE agent-scope counter and polls it
//                   (sc1 loads + s_sleep) until it reaches the generation's target --
//                   the barrier of mlp2_loop_kernel (csrc/mlp_fused.hip grid_sync);
//   kind 1 (xcd):   XCD-hierarchical: a workgroup adds to its XCD's counter (HW_REG_XCC_ID,
//                   its own 128-byte line, served by that XCD's L2 path); the last arriver
//                   of the XCD -- told by the value its add returned -- adds 1 to the top
//                   counter; every workgroup polls the top counter for 8 arrivals per
//                   generation;
//   kind 2 (empty): no barrier (the loop's own cost, subtracted by the tool).
// Each iteration also stores one word per workgroup write-through (the hand-off a real
// step publishes before its barrier).  Workgroup 0 stamps s_memrealtime at the start and
// after every 64th barrier.  Every wait is bounded (timeout -> err, every workgroup leaves).
#include "common.h"

namespace jdt {

__global__ void __launch_bounds__(512) barrier_lab_kernel(int kind, int iters, unsigned* ctr, int* err,
                                                          float* sink, unsigned long long* stamps,
                                                          long long timeout) {
  __shared__ int ok;
  const int b = blockIdx.x, G = gridDim.x;
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
  xcc &= 7u;
  // workgroups per XCD (round-robin dispatch: L % 8 -> XCD, checked by the host probe)
  const unsigned per_xcd = (unsigned)(G / 8 + ((int)(b % 8) < G % 8 ? 1 : 0));
  unsigned* flat = ctr;                // line 0
  unsigned* top = ctr + 32;            // line 1
  unsigned* mine = ctr + 32 * (2 + xcc);
  if (b == 0 && threadIdx.x == 0 && stamps) stamps[0] = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
    if (threadIdx.x == 0) __hip_atomic_store((__attribute__((address_space(1))) float*)(sink + b), (float)it,
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (kind == 2) continue;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      ok = 1;
      unsigned* poll;
      unsigned target;
      if (kind == 0) {
        __hip_atomic_fetch_add(flat, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        poll = flat;
        target = (unsigned)G * (unsigned)(it + 1);
      } else {
        const unsigned old = __hip_atomic_fetch_add(mine, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old % per_xcd == per_xcd - 1) __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        poll = top;
        target = 8u * (unsigned)(it + 1);
      }
      const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(poll, (short)0, 4, 0x00020000);
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while ((int)((unsigned)__builtin_amdgcn_raw_buffer_load_b32(r, 0, 0, 16) - target) < 0) {
        if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > timeout) {
          atomicOr(err, 1);
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
    if (!ok) break;
    if (b == 0 && threadIdx.x == 0 && stamps && (it + 1) % 64 == 0)
      stamps[(it + 1) / 64] = __builtin_amdgcn_s_memrealtime();
  }
}

// a trivial kernel: the boundary reference (back-to-back launches in one graph)
__global__ void __launch_bounds__(512) boundary_lab_kernel(float* sink) {
  if (threadIdx.x == 0) sink[blockIdx.x] += 1.f;
}

}  // namespace jdt
using namespace jdt;

// kind 0 / 1 / 2 (above); ctr: >= 10 * 32 zeroed words (monotonic within one launch; the
// caller zeroes them between launches); G workgroups (all resident: the caller checks).
JDT_API int jdt_barrier_lab(int kind, int G, int iters, unsigned* ctr, int* err, float* sink,
                            unsigned long long* stamps, long long timeout, void* stream) {
  if (kind < 0 || kind > 2 || G < 8 || G > 1024 || (G % 8) || iters < 1 || !ctr || !err || !sink) return -2;
  hipLaunchKernelGGL(barrier_lab_kernel, dim3(G), dim3(512), 0, static_cast<hipStream_t>(stream), kind, iters, ctr,
                     err, sink, stamps, timeout);
  return HIP_LAUNCH_CHECK();
}

JDT_API int jdt_boundary_lab(int G, float* sink, void* stream) {
  if (G < 1 || G > 1024 || !sink) return -2;
  hipLaunchKernelGGL(boundary_lab_kernel, dim3(G), dim3(512), 0, static_cast<hipStream_t>(stream), sink);
  return HIP_LAUNCH_CHECK();
}
