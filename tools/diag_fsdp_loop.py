"""Per-leaf gradient scale of the fused FSDP per-minibatch loop over xGMI (ranks sharing
one GPU) against the fp64 oracle: eager vs graph-replayed probe step."""
import functools
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tests import xgmi_workers as XW  # noqa: E402
from tests.oracle import mlp_grads_fp64  # noqa: E402
from tests.test_grad_scale_gpu import _batch, _load  # noqa: E402
from jax_distributed_tuts_amd.runtime.launch import spawn  # noqa: E402


def main():
    for ws in (1, 2, 4):
        for cap in (False, True):
            d = tempfile.mkdtemp()
            spawn(functools.partial(XW.grad_probe_xgmi, kind="fsdp_loop_sgd", capture=cap), ws, d, gpu=True)
            res = _load(d, "gpx_fsdp_loop_sgd", ws)
            b = _batch()
            want = mlp_grads_fp64(res[0]["before"], ["input_dense", "output_dense"], b.inputs, b.labels, n_mb=4)
            for r, o in enumerate(res):
                line = []
                for n in want:
                    g = (o["before"][n].double() - o["after"][n].double()).flatten()
                    w = want[n].double().flatten()
                    rel = float((g - w).norm() / w.norm())
                    sc = float(g @ w / (w @ w))
                    line.append(f"{n}: rel {rel:.4f} scale {sc:.4f}")
                print(f"ws={ws} capture={cap} rank {r}: " + "; ".join(line), flush=True)


if __name__ == "__main__":
    main()
