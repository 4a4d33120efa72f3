"""Where the in-epilogue AdamW and the plain AdamW pass differ on the LM (per leaf:
max |diff| and the count of elements apart > 1e-6), next to plain-vs-plain (the
step's run-to-run noise).  Usage: python tools/diag_lm_epi_adamw.py [--per-mb]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jax_distributed_tuts_amd.models.transformer import TransformerConfig  # noqa: E402
from jax_distributed_tuts_amd.parallel.pipeline_lm import build_lm_pipeline, lm_batch  # noqa: E402
from jax_distributed_tuts_amd.utils.train_state import Batch, adamw  # noqa: E402

DEV = torch.device("cuda", 0)
layer_major = "--per-mb" not in sys.argv


def run(fused):
    os.environ["JDT_LM_FUSED_OPT"] = fused
    tr, cfg = build_lm_pipeline(None, DEV, TransformerConfig(), num_microbatches=4, tx=adamw(3e-4),
                                layer_major_single_stage=layer_major)
    b = lm_batch(cfg, global_batch=16, seed=1)
    b = Batch(b.inputs.to(DEV), b.labels.to(DEV))
    for _ in range(3):
        tr.step(b)
    torch.cuda.synchronize()
    return tr.state.params


res = {k: run(f) for k, f in (("fused", "1"), ("plain", "0"), ("plain2", "0"))}
for a, b in (("fused", "plain"), ("plain2", "plain")):
    print(f"== {a} vs {b} (layer_major={layer_major})")
    Pa, Pb = res[a], res[b]
    for n in Pa.names():
        d = (Pa.p(n) - Pb.p(n)).abs()
        nd = int((d > 1e-6).sum())
        if nd:
            print(f"  {n:28s} max {float(d.max()):.3e}  n>1e-6 {nd}/{d.numel()}")
