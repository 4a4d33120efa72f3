// Host-side AddressSanitizer check of the kernel library's extern "C" entry points
// (SURVEY §5.2 "optional ASan builds of the C++ extension (host side)").
//
// Built by `python -m jax_distributed_tuts_amd.ops.build --asan-check`: every
// csrc/*.hip object is recompiled with `-Xarch_host -fsanitize=address` (device
// code unchanged -- GPU sanitizers are not used on this pool), linked with this
// driver and run on the CPU.  It exercises the host code that needs no GPU: the
// argument validation of every launcher (each rejects before touching the
// device), the struct-layout probes the ctypes mirrors check, the grouped-GEMM
// planner's early exits and the collectives' rank/world checks.  ASan aborts the
// run on any out-of-bounds / use-after-free in that code.
#include <cstdio>
#include <cstring>
#include <vector>

extern "C" {
int jdt_gemm_args_size();
int jdt_mlp2_args_size();
int jdt_md_args_size();
int jdt_xgmi_adam_size();
int jdt_xgmi_segs_size();
int jdt_gemm(const void* ga, int batch, int cfg, int splits, float* ws, long ws_floats, unsigned* counters,
             long n_counters, void* stream);
int jdt_gemm_group(const void* gs, int n, float* ws, long ws_floats, unsigned* counters, long n_counters,
                   void* stream);
int jdt_mlp2(const void* args, int phase, int k_in, int c, void* stream);
int jdt_md_layer(const void* args, int phase, int head, void* stream);
int jdt_xgmi_create(int rank, int world, long cap_floats, void** ctx_out, void* handles_out);
int jdt_p2p_create(int rank, int world, long slot_bytes, int n_slots, void** ctx_out, void* handles_out);
int jdt_adamw(float* p, float* g, float* m, float* v, void* shadow, long n, float lr, float b1, float b2, float eps,
              float wd, float grad_scale, int* step, unsigned* ticket, int zero_grad, void* stream);
int jdt_sgd(float* p, float* g, float* buf, void* shadow, long n, float lr, float momentum, float wd,
            float grad_scale, int* step, unsigned* ticket, int zero_grad, void* stream);
int jdt_colsum(const void* x, long ld, int M, int N, float* out, void* stream);
}

static int failures = 0;
#define EXPECT(cond, what)                                   \
  do {                                                       \
    if (!(cond)) {                                           \
      std::fprintf(stderr, "FAIL: %s\n", what);              \
      ++failures;                                            \
    }                                                        \
  } while (0)

int main() {
  // layout probes (the Python ctypes mirrors compare against these)
  EXPECT(jdt_gemm_args_size() > 0 && jdt_mlp2_args_size() > 0 && jdt_md_args_size() > 0, "struct sizes");
  EXPECT(jdt_xgmi_adam_size() > 0 && jdt_xgmi_segs_size() > 0, "xgmi struct sizes");

  // every launcher rejects bad arguments on the host, before any device call
  std::vector<unsigned char> gemm(jdt_gemm_args_size(), 0);
  EXPECT(jdt_gemm(gemm.data(), 1, -1, -1, nullptr, 0, nullptr, 0, nullptr) == 0, "gemm M = N = 0 is a no-op");
  EXPECT(jdt_gemm_group(gemm.data(), 0, nullptr, 0, nullptr, 0, nullptr) == 1, "empty group declined");
  std::vector<unsigned char> mlp2(jdt_mlp2_args_size(), 0);
  EXPECT(jdt_mlp2(mlp2.data(), 0, 784, 10, nullptr) == -3, "mlp2 rejects M = 0");
  EXPECT(jdt_mlp2(mlp2.data(), 0, 100, 10, nullptr) == -3, "mlp2 rejects an input width it is not built for");
  std::vector<unsigned char> md(jdt_md_args_size(), 0);
  EXPECT(jdt_md_layer(md.data(), 0, 0, nullptr) == -3, "md rejects N != 512");
  void* ctx = nullptr;
  unsigned char handles[3 * 64];
  EXPECT(jdt_xgmi_create(0, 1, 1024, &ctx, handles) == -4 && ctx == nullptr, "xgmi rejects world 1");
  EXPECT(jdt_xgmi_create(3, 2, 1024, &ctx, handles) == -4, "xgmi rejects rank >= world");
  EXPECT(jdt_xgmi_create(0, 9, 1024, &ctx, handles) == -4, "xgmi rejects world > 8");
  EXPECT(jdt_p2p_create(0, 1, 4096, 2, &ctx, handles) == -4, "p2p rejects world 1");
  EXPECT(jdt_p2p_create(0, 2, 4096, 0, &ctx, handles) == -2, "p2p rejects 0 slots");
  EXPECT(jdt_p2p_create(0, 2, 0, 2, &ctx, handles) == -2, "p2p rejects empty slots");
  EXPECT(jdt_adamw(nullptr, nullptr, nullptr, nullptr, nullptr, 0, 1e-3f, .9f, .999f, 1e-8f, 0.f, 1.f, nullptr,
                   nullptr, 1, nullptr) == 0, "adamw n = 0 is a no-op");
  float* mis = reinterpret_cast<float*>(reinterpret_cast<char*>(handles) + 4);  // misaligned
  EXPECT(jdt_adamw(mis, mis, mis, mis, nullptr, 16, 1e-3f, .9f, .999f, 1e-8f, 0.f, 1.f, nullptr, nullptr, 1,
                   nullptr) == -2, "adamw rejects misaligned buffers");
  EXPECT(jdt_sgd(nullptr, nullptr, nullptr, nullptr, 0, .1f, 0.f, 0.f, 1.f, nullptr, nullptr, 1, nullptr) == 0,
         "sgd n = 0 is a no-op");
  EXPECT(jdt_colsum(handles, 7, 4, 7, nullptr, nullptr) == -3, "colsum rejects N % 8");
  std::printf("asan host check: %d failure(s)\n", failures);
  return failures ? 1 : 0;
}
