"""jax_distributed_tuts_amd -- MI355X-native distributed-training tutorial framework.

Capabilities of AmanSwar/jax-distributed-tuts (DP with gradient accumulation,
FSDP/ZeRO-3 parameter sharding, GPipe pipeline parallelism and hybrid DP x PP,
a CPU multi-device simulation mode, named-scope tracing, (sum, count) metrics)
rebuilt on PyTorch-ROCm process groups (RCCL over xGMI) and hand-written
gfx950 HIP kernels.

Layout:
  ops/       HIP kernels (csrc/*.hip) + ctypes bindings + torch CPU references
  runtime/   process bootstrap, Mesh, CPU-simulation launcher
  comm/      JAX-named collectives over mesh axes (RCCL / gloo)
  models/    MLP classifiers, transformer, with explicit fused backward passes
  parallel/  dp.py, fsdp.py, pipeline.py (+ hybrid), sync_gradients
  utils/     TrainState, Batch, accumulation, metrics, rng folding, profiling
"""
__version__ = "0.1.0"
