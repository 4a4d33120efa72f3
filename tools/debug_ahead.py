"""Diagnostic: run-ahead backward launched eagerly, counters dumped after each launch."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jax_distributed_tuts_amd.models.mlp import Classifier  # noqa: E402
from jax_distributed_tuts_amd.parallel.dp import DataParallelTrainer, DPConfig, init_dp  # noqa: E402
from jax_distributed_tuts_amd.utils.train_state import Batch, adamw  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
b = Batch(torch.randn(128, 784, generator=g).to(dev), torch.randint(0, 10, (128,), generator=g).to(torch.int32).to(dev))
st = init_dp(Classifier(), adamw(1e-3), 69, dev)
tr = DataParallelTrainer(st, None, DPConfig(4, "kernel"))
tr.step(b)
eng = tr.fused
print("ahead_ok", eng.ahead_ok, flush=True)
for n in (1, 1, 2):
    eng.run_ahead(b, n)
    torch.cuda.synchronize()
    zt = eng.ztick.cpu()
    nb = 32
    print("line0", zt[:3].tolist(), "cols", zt[32:32 * (1 + nb)].view(nb, 32)[:, 0].tolist(), flush=True)
    print("tiles", zt[32 * (1 + nb):].view(8, 32)[:, :28].tolist(), flush=True)
    print("step", int(st.opt_state["count"].item()), flush=True)

# stamps of one more launch: per-workgroup start / partial stored / barrier passed / end
import ctypes  # noqa: E402

from jax_distributed_tuts_amd.ops import _lib  # noqa: E402

ah = type(eng._ahead_args)()
ctypes.memmove(ctypes.byref(ah), ctypes.byref(eng._ahead_args), ctypes.sizeof(ah))
sc = torch.zeros(224 * 16, dtype=torch.int64, device=dev)
ah.stamps = sc.data_ptr()
_lib.check(_lib.lib().jdt_mlp2(ctypes.byref(ah), 2, 784, 10, _lib.stream_ptr()), "bwd_ahead")
torch.cuda.synchronize()
S = sc.cpu().view(224, 16).double() * 0.01
t0 = S[:, 0].min()
order = torch.argsort(S[:, 0])
print("err after stamped launch", int(eng.ztick[1].item()))
for i in order.tolist()[:4] + order.tolist()[-8:]:
    print(f"wg {i:3d}: start {float(S[i, 0] - t0):9.2f} stored {float(S[i, 8] - t0):9.2f} "
          f"barrier {float(S[i, 9] - t0):9.2f} end {float(S[i, 4] - t0):9.2f}")
print("max barrier wait", float((S[:, 9] - S[:, 8]).max()), "us")
