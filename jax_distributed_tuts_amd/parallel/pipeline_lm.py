"""Transformer-LM pipeline construction (BASELINE config #5: 4-layer transformer,
hybrid DP=2 x PP=4).  Synthetic data: uniform random token sequences, labels =
inputs shifted by one (next-token prediction)."""
from __future__ import annotations

import torch

from ..models.transformer import TransformerConfig, TransformerLM, lm_stage
from ..runtime.dist import Mesh
from ..utils import rng as R
from ..utils.train_state import Batch, TrainState, adamw
from .pipeline import GPipeTrainer, PipeConfig, init_stage_params


def lm_batch(cfg: TransformerConfig, global_batch: int = 16, seed: int = 1) -> Batch:
    g = torch.Generator().manual_seed(seed)
    toks = torch.randint(0, cfg.vocab_size, (global_batch, cfg.seq_len + 1), generator=g, dtype=torch.int64)
    return Batch(toks[:, :-1].to(torch.int32).contiguous(), toks[:, 1:].to(torch.int32).contiguous())


def build_lm_pipeline(mesh: Mesh, dev, cfg: TransformerConfig = TransformerConfig(), num_microbatches: int = 4,
                      lr: float = 3e-4, seed: int = 0, comm: str = "auto", merge_single_stage: bool = False,
                      layer_major_single_stage: bool = True, tx=None, mb_streams=None, wpass_streams=None):
    S, s = (mesh.axis_size("pipe"), mesh.axis_index("pipe")) if mesh is not None else (1, 0)
    stage = lm_stage(cfg, S, s)
    full = TransformerLM(cfg)
    P = init_stage_params(stage, full.param_specs(), seed, dev)
    st = TrainState.create(apply_fn=stage, params=P, tx=tx if tx is not None else adamw(lr), rng=R.PRNGKey(seed))
    pc = PipeConfig(num_microbatches, comm=comm, merge_single_stage=merge_single_stage,
                    layer_major_single_stage=layer_major_single_stage)
    if mb_streams is not None:
        pc.mb_streams = int(mb_streams)
    if wpass_streams is not None:
        pc.wpass_streams = int(wpass_streams)
    return GPipeTrainer(st, mesh, pc), cfg
