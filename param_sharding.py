"""FSDP / ZeRO-3 training of the tutorial classifier (reference param_sharding.py).

    python param_sharding.py                        # every visible GPU, one rank each (RCCL / xGMI)
    torchrun --nproc-per-node 8 param_sharding.py   # the same under an external launcher
    python param_sharding.py --sim-cpu 8            # 8 gloo CPU ranks

Params, grads and AdamW moments are sharded with the reference rule
(min_weight_size = 2**4 as set at param_sharding.py:244-246); shard table in
SURVEY §2.7.  Schedule: 15 steps + 1 printed step "FSDP - Final metrics"
(param_sharding.py:389-397).
"""
from __future__ import annotations

import argparse

import torch

from data_paral import synthetic_batch
from jax_distributed_tuts_amd.models.mlp import Classifier
from jax_distributed_tuts_amd.parallel.dp import shard_batch
from jax_distributed_tuts_amd.parallel.fsdp import FSDPConfig, FSDPTrainer, init_fsdp
from jax_distributed_tuts_amd.runtime import dist as D
from jax_distributed_tuts_amd.runtime.dist import Mesh
from jax_distributed_tuts_amd.utils.config import fsdp_config
from jax_distributed_tuts_amd.utils.cli import add_common_args, entry_main, make_tx
from jax_distributed_tuts_amd.utils.metrics import print_metrics
from jax_distributed_tuts_amd.utils.train_state import Batch, get_num_params


def main(args):
    cfg = fsdp_config()
    cfg.model.num_layers = args.num_layers
    dev = D.device()
    axis = cfg.model.data_axis_name
    mesh = Mesh({axis: D.world_size()})
    model = Classifier.from_config(cfg.model)
    state = init_fsdp(model, make_tx(args, cfg.model.lr), cfg.seed, dev, mesh, axis, cfg.model.min_weight_size)
    batch = shard_batch(synthetic_batch(cfg, cfg.seed + 1), mesh, axis)
    batch = Batch(batch.inputs.to(dev), batch.labels.to(dev))
    tr = FSDPTrainer(state, mesh, FSDPConfig(cfg.num_minibatches, cfg.model.min_weight_size, axis,
                                             gather_once=args.gather_once or args.accum != "loop",
                                             scatter_once=args.scatter_once or args.accum != "loop",
                                             fused_kernels=args.accum == "kernel"))
    if D.rank() == 0:
        sp = state.extra["sharded"]
        print(f"[param_sharding] {mesh} global params={get_num_params(sp)} local flat={sp.local.numel} "
              f"sharded={sp.sharded_names} replicated={sp.repl_names}")
    for _ in range(args.steps):
        tr.step(batch)
    tr.metrics.zero_()
    tr.step(batch)
    tr.finalize()  # raises (non-zero exit) if an xGMI gather / reduce-scatter timed out
    if args.check_replication:
        from jax_distributed_tuts_amd.utils.debug import check_trainer_replication

        check_trainer_replication(tr)
    if D.rank() == 0:
        print_metrics(tr.metrics, "FSDP - Final metrics")


if __name__ == "__main__":
    ap = add_common_args(argparse.ArgumentParser(), steps=15, accum_choices=("loop", "fused", "kernel"))
    ap.add_argument("--gather-once", action="store_true")
    ap.add_argument("--scatter-once", action="store_true")
    a = ap.parse_args()
    entry_main(main, a, __file__)
