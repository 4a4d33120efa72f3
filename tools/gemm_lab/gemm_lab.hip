// GEMM main-loop lab (gfx950): which tile / MFMA shape / ring depth / split-K the
// transformer's mid-size GEMMs (M = 512 / 2048 tokens, N and K 512..2048) want.
// Standalone executable: C[M,N] (bf16) = A[M,K] . B[N,K]^T, both operands
// K-contiguous (the "mk x nk" layout), LDS-DMA (global_load_lds) ring with counted
// vmcnt + raw s_barrier, XOR-swizzled 128-byte row images, 32x32x16 or 16x16x32
// MFMA fragments, optional split-K with fp32 slabs combined by a second launch.
// Prints one line per (shape, config): us per launch (200 back-to-back launches,
// hipEvent), TF/s and the max relative error against a naive fp32 kernel.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o gemm_lab gemm_lab.hip && ./gemm_lab
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <vector>
#include <string.h>

typedef uint16_t bf16_t;
typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) { __bf16 b = (__bf16)f; return __builtin_bit_cast(bf16_t, b); }

constexpr int BK = 64;

template <int P, int LPW>
__device__ __forceinline__ void wait_bar(int pend) {
  if constexpr (P > 0) {
    if (pend >= P) {
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(P * LPW) : "memory");
      return;
    }
    wait_bar<P - 1, LPW>(pend);
  } else {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
}

// one [EXT][64] row image: EXT*128 bytes = EXT/8 wave-instructions of 1 KiB
template <int EXT, int NW>
__device__ __forceinline__ void stage(const bf16_t* src, long ld, int k0, bf16_t* img, int wid, int lane) {
  constexpr int IPW = EXT / (8 * NW);
  static_assert(IPW >= 1, "pieces");
#pragma unroll
  for (int i = 0; i < IPW; ++i) {
    const int ins = wid * IPW + i;
    const int r = ins * 8 + (lane >> 3), c = (lane & 7) ^ (r & 7);
    const bf16_t* gp = src + (long)r * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gp,
                                     (__attribute__((address_space(3))) void*)(img + ins * 512), 16, 0, 0);
  }
}

// 32x32x16 fragment: lane l -> row base + (l & 31), k = kk + 8 (l >> 5) .. +7
__device__ __forceinline__ bf16x8 frag32(const bf16_t* img, int base, int kk, int lane) {
  const int r = base + (lane & 31), c = (kk >> 3) + (lane >> 5);
  return *reinterpret_cast<const bf16x8*>(img + r * BK + ((c ^ (r & 7)) << 3));
}
// 16x16x32 fragment: lane l -> row base + (l & 15), k = kk + 8 (l >> 4) .. +7
__device__ __forceinline__ bf16x8 frag16(const bf16_t* img, int base, int kk, int lane) {
  const int r = base + (lane & 15), c = (kk >> 3) + (lane >> 4);
  return *reinterpret_cast<const bf16x8*>(img + r * BK + ((c ^ (r & 7)) << 3));
}

// MF = 32: v_mfma_f32_32x32x16_bf16, MF = 16: v_mfma_f32_16x16x32_bf16
template <int BM, int BN, int WM, int WN, int S, int MF>
__global__ void __launch_bounds__(64 * WM * WN) lab_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                            bf16_t* __restrict__ C, float* __restrict__ slab, int M,
                                                            int N, int K, int splits) {
  constexpr int NW = WM * WN;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / MF, TN = WTN / MF;
  constexpr int STAGE = (BM + BN) * BK;
  constexpr int LPW = (BM + BN) / (8 * NW);
  static_assert((S - 2) * LPW <= 63, "vmcnt");
  __shared__ __attribute__((aligned(16))) bf16_t smem[S * STAGE];
  const int tiles_n = N / BN;
  const int nwg = gridDim.x;
  int bid = blockIdx.x;
  {
    const int xcd = bid % 8, q = nwg / 8, rr = nwg % 8;
    bid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
  }
  const int tm0 = (bid / tiles_n) * BM, tn0 = (bid % tiles_n) * BN;
  const int split = blockIdx.y, kchunk = K / splits, kbeg = split * kchunk;
  const int nkt = kchunk / BK;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wm = wid / WN, wn = wid % WN;
  const bf16_t* Ab = A + (long)tm0 * K;
  const bf16_t* Bb = B + (long)tn0 * K;
  using acc_t = typename std::conditional<MF == 32, f32x16, f32x4>::type;
  acc_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < (MF == 32 ? 16 : 4); ++e) acc[i][j][e] = 0.f;
  auto issue = [&](int kt) {
    bf16_t* st = smem + (kt % S) * STAGE;
    const int k0 = kbeg + kt * BK;
    stage<BM, NW>(Ab, K, k0, st, wid, lane);
    stage<BN, NW>(Bb, K, k0, st + BM * BK, wid, lane);
  };
#pragma unroll
  for (int s = 0; s < S - 1; ++s)
    if (s < nkt) issue(s);
  for (int kt = 0; kt < nkt; ++kt) {
    wait_bar<S - 2, LPW>(min(S - 2, nkt - 1 - kt));
    if (kt + S - 1 < nkt) issue(kt + S - 1);
    const bf16_t* As = smem + (kt % S) * STAGE;
    const bf16_t* Bs = As + BM * BK;
    if constexpr (MF == 32) {
#pragma unroll
      for (int kk = 0; kk < BK; kk += 16) {
        bf16x8 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = frag32(As, wm * WTM + i * 32, kk, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[j] = frag32(Bs, wn * WTN + j * 32, kk, lane);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < BK; kk += 32) {
        bf16x8 af[TM], bfr[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) af[i] = frag16(As, wm * WTM + i * 16, kk, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[j] = frag16(Bs, wn * WTN + j * 16, kk, lane);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
  }
  // epilogue: plain stores (bf16 C, or fp32 slab when split)
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if constexpr (MF == 32) {
        const int col = tn0 + wn * WTN + j * 32 + (lane & 31);
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int row = tm0 + wm * WTM + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
          if (splits > 1) slab[((long)split * M + row) * N + col] = acc[i][j][e];
          else C[(long)row * N + col] = f2bf(acc[i][j][e]);
        }
      } else {
        const int col = tn0 + wn * WTN + j * 16 + (lane & 15);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = tm0 + wm * WTM + i * 16 + (lane >> 4) * 4 + e;
          if (splits > 1) slab[((long)split * M + row) * N + col] = acc[i][j][e];
          else C[(long)row * N + col] = f2bf(acc[i][j][e]);
        }
      }
    }
}

__global__ void combine_kernel(const float* __restrict__ slab, bf16_t* __restrict__ C, long MN, int splits) {
  const long i = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= MN) return;
  float4 s = *reinterpret_cast<const float4*>(slab + i);
  for (int p = 1; p < splits; ++p) {
    const float4 t = *reinterpret_cast<const float4*>(slab + p * MN + i);
    s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
  }
  C[i] = f2bf(s.x); C[i + 1] = f2bf(s.y); C[i + 2] = f2bf(s.z); C[i + 3] = f2bf(s.w);
}

__global__ void ref_kernel(const bf16_t* A, const bf16_t* B, float* R, int M, int N, int K) {
  const int row = blockIdx.y, col = blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= N) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += bf2f(A[(long)row * K + k]) * bf2f(B[(long)col * K + k]);
  R[(long)row * N + col] = s;
}

__global__ void fill_kernel(bf16_t* p, long n, unsigned seed) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned x = (unsigned)i * 2654435761u ^ seed;
  x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
  p[i] = f2bf(((x & 0xffff) / 32768.f - 1.f));
}

struct Bufs { bf16_t *A, *B, *C; float *R, *slab; };

template <int BM, int BN, int WM, int WN, int S, int MF>
void run(const char* name, const Bufs& b, int M, int N, int K, int splits) {
  if (M % BM || N % BN || (K / splits) % BK || K % splits) return;
  auto kfn = lab_kernel<BM, BN, WM, WN, S, MF>;
  dim3 grid((M / BM) * (N / BN), splits);
  const long MN = (long)M * N;
  auto launch = [&]() {
    hipLaunchKernelGGL(kfn, grid, dim3(64 * WM * WN), 0, 0, b.A, b.B, b.C, b.slab, M, N, K, splits);
    if (splits > 1) hipLaunchKernelGGL(combine_kernel, dim3((MN / 4 + 255) / 256), dim3(256), 0, 0, b.slab, b.C, MN, splits);
  };
  launch();
  CK(hipDeviceSynchronize());
  // check
  std::vector<bf16_t> hc(MN);
  std::vector<float> hr(MN);
  CK(hipMemcpy(hc.data(), b.C, MN * 2, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hr.data(), b.R, MN * 4, hipMemcpyDeviceToHost));
  double mx = 0, ref = 0;
  for (long i = 0; i < MN; ++i) {
    uint32_t u = ((uint32_t)hc[i]) << 16; float c; memcpy(&c, &u, 4);
    mx = fmax(mx, fabs(c - hr[i]));
    ref = fmax(ref, fabs(hr[i]));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int R = 200;
  for (int i = 0; i < 20; ++i) launch();
  CK(hipEventRecord(e0));
  for (int i = 0; i < R; ++i) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / R;
  printf("%-22s %5d %5d %5d split %d grid %5d : %8.2f us %7.1f TF/s  err %.2e\n", name, M, N, K, splits,
         (M / BM) * (N / BN) * splits, us, 2.0 * M * N * K / us / 1e6, mx / (ref + 1e-9));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
  const int shapes[][3] = {{512, 2048, 512}, {512, 512, 2048}, {2048, 2048, 512}, {2048, 512, 2048}, {2048, 1536, 512},
                           {512, 1536, 512}};
  const long maxe = 2048L * 2048;
  Bufs b;
  CK(hipMalloc(&b.A, maxe * 2));
  CK(hipMalloc(&b.B, maxe * 2));
  CK(hipMalloc(&b.C, maxe * 2));
  CK(hipMalloc(&b.R, maxe * 4));
  CK(hipMalloc(&b.slab, maxe * 4 * 8));
  hipLaunchKernelGGL(fill_kernel, dim3(maxe / 256), dim3(256), 0, 0, b.A, maxe, 1u);
  hipLaunchKernelGGL(fill_kernel, dim3(maxe / 256), dim3(256), 0, 0, b.B, maxe, 7u);
  for (auto& s : shapes) {
    const int M = s[0], N = s[1], K = s[2];
    hipLaunchKernelGGL(ref_kernel, dim3((N + 255) / 256, M), dim3(256), 0, 0, b.A, b.B, b.R, M, N, K);
    CK(hipDeviceSynchronize());
    run<32, 32, 2, 2, 3, 16>("32x32 w4 S3 m16", b, M, N, K, 1);
    run<64, 64, 2, 2, 3, 16>("64x64 w4 S3 m16", b, M, N, K, 1);
    run<64, 64, 2, 2, 3, 32>("64x64 w4 S3 m32", b, M, N, K, 1);
    run<64, 64, 2, 2, 4, 32>("64x64 w4 S4 m32", b, M, N, K, 1);
    run<64, 64, 2, 2, 6, 32>("64x64 w4 S6 m32", b, M, N, K, 1);
    run<64, 64, 2, 2, 8, 32>("64x64 w4 S8 m32", b, M, N, K, 1);
    run<128, 64, 2, 2, 3, 32>("128x64 w4 S3 m32", b, M, N, K, 1);
    run<128, 64, 2, 2, 4, 32>("128x64 w4 S4 m32", b, M, N, K, 1);
    run<64, 128, 2, 2, 4, 32>("64x128 w4 S4 m32", b, M, N, K, 1);
    run<128, 128, 2, 2, 3, 32>("128x128 w4 S3 m32", b, M, N, K, 1);
    run<128, 128, 2, 2, 4, 32>("128x128 w4 S4 m32", b, M, N, K, 1);
    run<128, 128, 4, 2, 4, 32>("128x128 w8 S4 m32", b, M, N, K, 1);
    run<128, 128, 2, 2, 4, 32>("128x128 w4 S4 m32", b, M, N, K, 2);
    run<128, 128, 2, 2, 4, 32>("128x128 w4 S4 m32", b, M, N, K, 4);
    run<64, 64, 2, 2, 4, 32>("64x64 w4 S4 m32", b, M, N, K, 2);
    run<64, 64, 2, 2, 4, 32>("64x64 w4 S4 m32", b, M, N, K, 4);
    run<256, 128, 4, 2, 3, 32>("256x128 w8 S3 m32", b, M, N, K, 1);
    run<256, 128, 4, 2, 3, 32>("256x128 w8 S3 m32", b, M, N, K, 4);
  }
  return 0;
}
