"""The overlapped data-axis sync's bucket plan (parallel/pipeline.py
GPipeTrainer._sync_buckets over models/transformer.py TransformerLM.sync_groups): for
every stage of 1-, 2- and 4-stage LM pipelines the buckets tile the optimizer range
[0, numel) exactly once, each starts 4-aligned (the xGMI kernel's bucket rule), every
parameter falls in the bucket of the W-pass GEMM that finalises it (a weight in its
own GEMM's bucket; biases / LayerNorm -- computed by the backward chain -- beside the
weight they follow), the metric slots ride on the bucket that ends the flat buffer,
exactly the last bucket issued advances the step counter, and the issue order is the
order the W pass runs its GEMMs (embedding first: final when the chain ends).
Host-only: the plan is pure index arithmetic."""
import types

import pytest

from jax_distributed_tuts_amd.models.transformer import TransformerConfig, lm_stage
from jax_distributed_tuts_amd.parallel.pipeline import GPipeTrainer
from jax_distributed_tuts_amd.utils.flat import FlatParams


def _owner(name: str) -> str:
    """The bucket key a parameter must land in."""
    if name.startswith("embed/"):
        return "embed"
    if name.startswith(("ln_f/", "head/")):
        return "head/kernel"
    b, rest = name.split("/", 1)
    if rest.startswith(("ln1/", "attn/qkv/")):
        return f"{b}/attn/qkv/kernel"
    if rest.startswith(("attn/out/", "ln2/")):
        return f"{b}/attn/out/kernel"
    return f"{b}/{rest.rsplit('/', 1)[0]}/kernel"   # mlp/fc1/*, mlp/fc2/*


@pytest.mark.parametrize("S", [1, 2, 4])
def test_buckets_tile_the_stage(S):
    cfg = TransformerConfig(vocab_size=512, d_model=128, n_heads=2, d_ff=256, seq_len=64, n_layers=4)
    for s in range(S):
        model = lm_stage(cfg, S, s)
        P = FlatParams(model.param_specs())
        fake = types.SimpleNamespace(state=types.SimpleNamespace(params=P), model=model, _buckets=None)
        b = GPipeTrainer._sync_buckets(fake)
        keys = [x[0] for x in b]
        # issue order == the W pass's GEMM order (weights_grads_of over head, layers top-down)
        wpass = [n for part in (["head"] if model.has_head else []) + list(reversed(list(model.layers)))
                 for n in ([f"head/kernel"] if part == "head" else
                           [f"block_{part}/mlp/fc2/kernel", f"block_{part}/mlp/fc1/kernel",
                            f"block_{part}/attn/out/kernel", f"block_{part}/attn/qkv/kernel"])]
        assert keys == (["embed"] if model.has_embed else []) + wpass, (S, s)
        spans = sorted((lo, hi) for _, lo, hi, _, _ in b)
        assert spans[0][0] == 0 and spans[-1][1] == P.numel
        assert all(a[1] == c[0] for a, c in zip(spans, spans[1:])), spans
        assert all(lo % 4 == 0 and hi > lo for lo, hi in spans)
        for name, (off, shape) in P.offsets.items():
            n = 1
            for d in shape:
                n *= d
            lo, hi = next((lo, hi) for k, lo, hi, _, _ in b if k == _owner(name))
            assert lo <= off and off + n <= hi, (name, _owner(name))
        # metrics on the bucket that ends at numel; one advance, on the last issued bucket
        assert [m for _, _, hi, m, _ in b] == [hi == P.numel for _, _, hi, _, _ in b]
        assert [a for *_, a in b] == [False] * (len(b) - 1) + [True]
