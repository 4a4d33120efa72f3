"""The overlapped data-axis sync's bucket plan (parallel/pipeline.py
GPipeTrainer._sync_buckets): for every stage of 1-, 2- and 4-stage LM pipelines the
buckets tile the optimizer range [0, numel) exactly once, each bucket is one whole
part (embedding / layer / head) starting 4-aligned (the xGMI kernel's bucket rule),
the metric slots ride on the bucket that ends the flat buffer, exactly the last bucket
issued advances the step counter, and the issue order is the order the W pass
finishes the parts (embedding first: its gradient is final when the chain ends; then
the head and the layers top-down).  Host-only: the plan is pure index arithmetic."""
import types

import pytest

from jax_distributed_tuts_amd.models.transformer import TransformerConfig, lm_stage
from jax_distributed_tuts_amd.parallel.pipeline import GPipeTrainer
from jax_distributed_tuts_amd.utils.flat import FlatParams


@pytest.mark.parametrize("S", [1, 2, 4])
def test_buckets_tile_the_stage(S):
    cfg = TransformerConfig(vocab_size=512, d_model=128, n_heads=2, d_ff=256, seq_len=64, n_layers=4)
    for s in range(S):
        model = lm_stage(cfg, S, s)
        P = FlatParams(model.param_specs())
        fake = types.SimpleNamespace(state=types.SimpleNamespace(params=P), model=model, _buckets=None)
        b = GPipeTrainer._sync_buckets(fake)
        parts = [x[0] for x in b]
        want = (["embed"] if model.has_embed else []) + (["head"] if model.has_head else []) \
            + list(reversed(list(model.layers)))
        assert parts == want, (S, s)
        spans = sorted((lo, hi) for _, lo, hi, _, _ in b)
        assert spans[0][0] == 0 and spans[-1][1] == P.numel
        assert all(a[1] == c[0] for a, c in zip(spans, spans[1:])), spans
        assert all(lo % 4 == 0 and hi > lo for lo, hi in spans)
        # every parameter lies inside the bucket of its own part
        for name, (off, shape) in P.offsets.items():
            part = "embed" if name.startswith("embed/") else (
                "head" if name.startswith(("ln_f/", "head/")) else int(name.split("/")[0].split("_")[1]))
            lo, hi = next((lo, hi) for p, lo, hi, _, _ in b if p == part)
            n = 1
            for d in shape:
                n *= d
            assert lo <= off and off + n <= hi, (name, part)
        # metrics on the bucket that ends at numel; one advance, on the last issued bucket
        assert [m for _, _, hi, m, _ in b] == [hi == P.numel for _, _, hi, _, _ in b]
        assert [a for *_, a in b] == [False] * (len(b) - 1) + [True]
