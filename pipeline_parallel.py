"""GPipe pipeline parallelism and hybrid DP x PP (the reference's
pipeline_parallel.py is an imports-only stub; this is the intended tutorial,
SURVEY §3.5).

    python pipeline_parallel.py --gpus 8                               # 8-stage MLP (BASELINE config #4)
    python pipeline_parallel.py --gpus 8 --dp 2 --model transformer    # DP=2 x PP=4 (config #5)
    torchrun --nproc-per-node 8 pipeline_parallel.py                   # the same under an external launcher
    python pipeline_parallel.py --sim-cpu 4 --dp 2                     # gloo CPU simulation

Default model: an MLP 784 -> 512 x 8 -> 10 (9 Dense layers, SiLU, dropout 0.1)
split over the pipe axis; 10 steps + 1 printed step.
"""
from __future__ import annotations

import argparse

import torch

from data_paral import synthetic_batch
from jax_distributed_tuts_amd.parallel.dp import shard_batch
from jax_distributed_tuts_amd.parallel.pipeline import GPipeTrainer, PipeConfig, init_stage_params, mlp_stage
from jax_distributed_tuts_amd.models.mlp import MLP
from jax_distributed_tuts_amd.runtime import dist as D
from jax_distributed_tuts_amd.runtime.dist import Mesh
from jax_distributed_tuts_amd.utils import rng as R
from jax_distributed_tuts_amd.utils.cli import add_common_args, entry_main, make_tx
from jax_distributed_tuts_amd.utils.config import dp_config
from jax_distributed_tuts_amd.utils.metrics import print_metrics
from jax_distributed_tuts_amd.utils.train_state import Batch, TrainState, adamw


def pp_mlp_dims(cfg, n_hidden_layers: int):
    return [cfg.data.input_size] + [cfg.model.hidden_size] * n_hidden_layers + [cfg.data.num_classes]


def build_mlp_pipeline(cfg, mesh, dev, n_hidden_layers=8, dropout_rate=None, num_microbatches=4, comm="auto",
                       merge_single_stage=False, tx=None):
    dims = pp_mlp_dims(cfg, n_hidden_layers)
    S, s = mesh.axis_size("pipe"), mesh.axis_index("pipe")
    dr = cfg.model.dropout_rate if dropout_rate is None else dropout_rate
    stage = mlp_stage(dims, S, s, dropout_rate=dr)
    full = MLP(dims, dropout_rate=dr)
    P = init_stage_params(stage, full.param_specs(), cfg.seed, dev)
    tx = tx if tx is not None else adamw(cfg.optimizer.learning_rate)
    st = TrainState.create(apply_fn=stage, params=P, tx=tx, rng=R.PRNGKey(cfg.seed))
    tr = GPipeTrainer(st, mesh, PipeConfig(num_microbatches, comm=comm, merge_single_stage=merge_single_stage))
    return tr


def main(args):
    cfg = dp_config()
    dev = D.device()
    ws = D.world_size()
    dp = args.dp
    mesh = Mesh({"data": dp, "pipe": ws // dp})
    if args.microbatches is None:
        from jax_distributed_tuts_amd.parallel.pipeline import default_microbatches

        args.microbatches = default_microbatches(ws // dp)
    if args.model == "transformer":
        from jax_distributed_tuts_amd.parallel.pipeline_lm import build_lm_pipeline, lm_batch

        tr, lm_cfg = build_lm_pipeline(mesh, dev, num_microbatches=args.microbatches)
        batch = shard_batch(lm_batch(lm_cfg, seed=1), mesh, "data")
    else:
        tr = build_mlp_pipeline(cfg, mesh, dev, args.hidden_layers, num_microbatches=args.microbatches,
                                tx=make_tx(args, cfg.optimizer.learning_rate))
        batch = shard_batch(synthetic_batch(cfg, cfg.seed + 1), mesh, "data")
    batch = Batch(batch.inputs.to(dev), batch.labels.to(dev))
    if D.rank() == 0:
        print(f"[pipeline_parallel] {mesh} model={args.model} stage0 params={tr.state.params.num_params()}")
    for _ in range(args.steps):
        tr.step(batch)
    tr.metrics.zero_()
    tr.step(batch)
    if hasattr(tr, "finalize"):
        tr.finalize()
    if args.check_replication:
        from jax_distributed_tuts_amd.utils.debug import check_trainer_replication

        check_trainer_replication(tr)
    m = tr.gather_metrics()
    if D.rank() == 0:
        print_metrics(m, f"PP{mesh.axis_size('pipe')} x DP{dp} - Final metrics")


if __name__ == "__main__":
    ap = add_common_args(argparse.ArgumentParser(), steps=10, accum_choices=("loop",))
    ap.add_argument("--dp", type=int, default=1)
    ap.add_argument("--microbatches", type=int, default=None,
                    help="GPipe microbatches (default: pipeline.default_microbatches, measured per stage count)")
    ap.add_argument("--hidden-layers", type=int, default=8)
    ap.add_argument("--model", choices=["mlp", "transformer"], default="mlp")
    a = ap.parse_args()
    entry_main(main, a, __file__)
