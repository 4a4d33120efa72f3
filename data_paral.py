"""Data-parallel training of the tutorial classifier (reference data_paral.py).

    python data_paral.py                       # DP over every visible GPU (one rank per GPU, RCCL/xGMI)
    python data_paral.py --gpus 1              # one GPU
    torchrun --nproc-per-node 8 data_paral.py  # the same 8-rank job under an external launcher
    python data_paral.py --sim-cpu 8           # 8 gloo CPU ranks (reference's simulated devices)
    python data_paral.py --accum kernel        # whole-step fused HIP kernels
    python data_paral.py --profile             # same run under rocprofv3 --pmc (counters + kernel stats)
    python data_paral.py --check-replication   # verify replicated params are bitwise equal on every rank

Schedule as the reference (data_paral.py:271-277): 10 training steps with
metrics accumulated, then one step on fresh metrics printed under "dp".
Config values verbatim from data_paral.py:38-72 (see utils/config.py).
"""
from __future__ import annotations

import argparse

import torch

from jax_distributed_tuts_amd.models.mlp import Classifier
from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp, shard_batch
from jax_distributed_tuts_amd.runtime import dist as D
from jax_distributed_tuts_amd.runtime.dist import Mesh
from jax_distributed_tuts_amd.utils.cli import add_common_args, entry_main, make_tx
from jax_distributed_tuts_amd.utils.config import dp_config
from jax_distributed_tuts_amd.utils.metrics import print_metrics
from jax_distributed_tuts_amd.utils.train_state import Batch, get_num_params


def synthetic_batch(cfg, seed: int) -> Batch:
    """data_paral.py:113-124 with B3 fixed: N(0,1) inputs, integer labels in [0, classes)."""
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(cfg.data.batch_size, cfg.data.input_size, generator=g)
    y = torch.randint(0, cfg.data.num_classes, (cfg.data.batch_size,), generator=g, dtype=torch.int64)
    return Batch(x, y.to(torch.int32))


def main(args):
    cfg = dp_config()
    cfg.model.num_layers = args.num_layers
    dev = D.device()
    mesh = Mesh({"data": D.world_size()})
    model = Classifier.from_config(cfg.model)
    state = init_dp(model, make_tx(args, cfg.optimizer.learning_rate), cfg.seed, dev, mesh)
    batch = shard_batch(synthetic_batch(cfg, cfg.seed + 1), mesh, "data")
    batch = Batch(batch.inputs.to(dev), batch.labels.to(dev))
    trainer = DataParallelTrainer(state, mesh, DPConfig(cfg.optimizer.num_minibatches, args.accum, comm=args.comm))
    if D.rank() == 0:
        print(f"[data_paral] {mesh} params={get_num_params(state)} device={dev} comm={trainer.comm_backend}")
    for _ in range(args.steps):
        trainer.step(batch)
    trainer.metrics.zero_()
    trainer.step(batch)
    trainer.finalize()
    if args.check_replication:
        from jax_distributed_tuts_amd.utils.debug import check_trainer_replication

        check_trainer_replication(trainer)
    if D.rank() == 0:
        print_metrics(trainer.metrics, "dp")


if __name__ == "__main__":
    ap = add_common_args(argparse.ArgumentParser(), steps=10)
    ap.add_argument("--comm", choices=["auto", "xgmi", "rccl"], default="auto",
                    help="N>1 gradient all-reduce: direct xGMI P2P kernel (+fused AdamW) or RCCL")
    a = ap.parse_args()
    if a.use_scan:
        a.accum = "scan"
    entry_main(main, a, __file__)
