"""Fused per-layer kernels as GPipe stage compute (csrc/mlp_deep.hip).

A GPipe stage of the tutorial MLPs (BASELINE config #4: 784 -> 512 x 8 -> 10,
split over the pipe axis) is a contiguous run of 512-wide SiLU/dropout Dense
layers, possibly starting with the 784-input layer (stage 0) and possibly
ending with the 10-class head (last stage).  The generic stage compute
(models/mlp.py) issues per microbatch one GEMM per layer forward, the CE
kernel, and a grouped dW+dX launch per layer backward.  Here every hidden
layer is ONE ``md_fwd`` and ONE ``md_bwd`` launch per microbatch:

* forward: GEMM + bias + SiLU + dropout, the backward factor
  G = silu'(Z) * mask / keep, the layer input transposed for the dW MFMA and --
  last stage -- the head's logits (fp32 atomics);
* backward: dZ of the layer from (a) the softmax-CE of the logits through the
  head (last stage's top layer), (b) dZ_{l+1} W_{l+1}^T (inner layers) or
  (c) the gradient the next stage sent, times G (stage-boundary variant), then
  dW / db (and the head's dW / db + metric slots) ACCUMULATED into the stage's
  grad buffer (mode 0 + ``accumulate``: microbatch accumulation, reference
  util.py:69-77);
* a non-first stage sends dX = dZ_0 W_0^T back with one GEMM launch.

Dropout streams equal the generic path's (offset (mb << 16) + (layer << 1),
step << 32, 4-row groups over the microbatch's rows), so both paths train the
same model (tests/test_fused_stage_gpu.py).  The optimizer (or the xGMI
all-reduce with fused AdamW) runs after the last microbatch, as before.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional

import torch

from ..ops import _lib
from ..ops import kernels as K
from .fused_mlp import DEEP_H, MdArgs

H = DEEP_H
C_HEAD = 10


def stage_supported(model, rows: int, device) -> bool:
    """A stage of a 784 -> 512 x k -> 10 SiLU MLP, microbatch rows <= 128, on GPU."""
    from ..models.mlp import MLP

    if torch.device(device).type != "cuda" or not isinstance(model, MLP) or model.act != "silu":
        return False
    if not (0 < rows <= 128) or model.dims[0] not in (784, H):
        return False
    hidden_out = model.dims[1:] if model.final_act else model.dims[1:-1]
    if not hidden_out or any(d != H for d in hidden_out):
        return False
    if not model.final_act:
        # last stage: the head (H -> 10) is fused into the last hidden layer's kernels
        # (784- or 512-wide input)
        if model.dims[-1] != C_HEAD or model.L < 2:
            return False
    return True


class FusedMLPStage:
    """Microbatch forward / backward of one pipeline stage on the md kernels.

    ``params``: the stage's FlatParams; ``n_mb`` microbatches of ``mb`` rows;
    ``step``: the device step counter (dropout offset; advanced by the optimizer)."""

    def __init__(self, model, params, n_mb: int, mb: int, step: torch.Tensor, seed: int,
                 mb_shift: int = 16, step_mul: int = 1, n_sets: int = 1):
        """``mb_shift`` / ``step_mul``: microbatch i, layer l draws dropout stream
        offset (i << mb_shift) + (l << 1) at counter high word step * step_mul -- the
        GPipe convention (16, 1) or the DP minibatch loop's (32, n_minibatches).
        ``n_sets`` > 1: microbatch i accumulates its grads / metric slots into set
        i % n_sets (set 0 = the params' grad buffer, the others private zeroed copies)
        and uses that set's dZ buffers, so the sets' microbatches may run on
        concurrent streams (every grad write is a read-modify-write); ``merge`` folds
        the private sets into the grad buffer afterwards."""
        self.model, self.P = model, params
        self.n_sets = max(1, int(n_sets))
        self.gx = [torch.zeros_like(params.grad) for _ in range(self.n_sets - 1)]
        self.n_mb, self.mb = n_mb, mb
        self.step, self.seed = step, seed & 0xFFFFFFFF
        self.mb_shift, self.step_mul = mb_shift, step_mul
        self.last = not model.final_act
        self.nh = model.L - 1 if self.last else model.L          # hidden layers run by md kernels
        self.k0 = model.dims[0]
        dev = params.master.device
        bf = dict(dtype=torch.bfloat16, device=dev)
        mp = (mb + 31) // 32 * 32
        self.ldint = mp
        # per microbatch and layer: backward factor, activation, transposed input (zero tail)
        self.G = [[torch.zeros((mb + 15) // 16 * 4, H, 4, dtype=torch.float32, device=dev) for _ in range(self.nh)]
                  for _ in range(n_mb)]
        self.Hs = [[torch.empty(mb, H, **bf) for _ in range(self.nh)] for _ in range(n_mb)]
        self.INT = [[torch.zeros(model.dims[l], mp, **bf) for l in range(self.nh)] for _ in range(n_mb)]
        # logits accumulators per microbatch, both step parities (md_bwd re-arms the other)
        self.logits = [torch.zeros(2, mb, C_HEAD, dtype=torch.float32, device=dev) for _ in range(n_mb)] \
            if self.last else None
        from .fused_mlp import deterministic

        self.det_logits = [torch.zeros(H // 16, mb, C_HEAD, dtype=torch.float32, device=dev) for _ in range(n_mb)] \
            if (self.last and deterministic()) else None
        # dZ of each layer (consumed by the launch of the layer below, then dead)
        self.dZs = [[torch.empty(mb, H, **bf) for _ in range(self.nh)] for _ in range(self.n_sets)]
        self.dZ = self.dZs[0]
        self.dX = [torch.empty(mb, self.k0, **bf) for _ in range(n_mb)]   # in flight to the previous stage
        self.kn = [f"{n}/kernel" for n in model.names]
        self.bn = [f"{n}/bias" for n in model.names]
        self._fwd: List[List[Optional[MdArgs]]] = [[None] * self.nh for _ in range(n_mb)]
        self._bwd: List[List[Optional[MdArgs]]] = [[None] * self.nh for _ in range(n_mb)]
        self._keys = [[None] * self.nh for _ in range(n_mb)]
        if _lib.lib().jdt_md_args_size() != ctypes.sizeof(MdArgs):
            raise RuntimeError("MdArgs layout mismatch")

    # ------------------------------------------------------------------ args
    def _g(self, i: int, name: str) -> int:
        """Address of leaf ``name``'s gradient in microbatch i's grad set."""
        g = self.P.g(name)
        k = i % self.n_sets
        return g.data_ptr() if k == 0 else self.gx[k - 1].data_ptr() + (g.data_ptr() - self.P.grad.data_ptr())

    def merge(self):
        """grad += every private set (then re-zeroed): after the sets' streams joined."""
        for g in self.gx:
            self.P.grad.add_(g)
            g.zero_()

    def _base(self, i: int, l: int, x_ptr: int) -> MdArgs:
        P, m = self.P, self.model
        a = MdArgs()
        a.M, a.K, a.N, a.C = self.mb, m.dims[l], H, C_HEAD
        a.inv_mb = 1.0 / self.mb
        a.X = x_ptr
        a.Ws0 = a.Ws1 = P.s(self.kn[l]).data_ptr()
        a.bs = P.s(self.bn[l]).data_ptr()
        a.G, a.Hout = self.G[i][l].data_ptr(), self.Hs[i][l].data_ptr()
        a.INT, a.ldint = self.INT[i][l].data_ptr(), self.ldint
        if self.last:
            hk, hb = self.kn[-1], self.bn[-1]
            a.Wh0 = a.Wh1 = P.s(hk).data_ptr()
            a.bh = P.s(hb).data_ptr()
            a.logits = self.logits[i].data_ptr()
            if self.det_logits is not None:
                a.det_logits = self.det_logits[i].data_ptr()
            a.gWh, a.gbh = self._g(i, hk), self._g(i, hb)
        a.keep = 1.0 - m.dropout_rate
        a.seed = self.seed
        a.offset = (i << self.mb_shift) + ((m.layer_id_base + l) << 1)
        a.step_mul = self.step_mul
        a.step = self.step.data_ptr()
        a.advance_step = 0
        a.fuse_opt = 0
        a.accumulate = 1
        a.mb_rows = 0
        a.gW, a.gb = self._g(i, self.kn[l]), self._g(i, self.bn[l])
        ms = P.metrics_slot
        a.mslot = ms.data_ptr() if i % self.n_sets == 0 else \
            self.gx[i % self.n_sets - 1].data_ptr() + (ms.data_ptr() - P.grad.data_ptr())
        return a

    # ------------------------------------------------------------------ passes
    def forward(self, i: int, x: torch.Tensor) -> Optional[torch.Tensor]:
        """Microbatch i: x [mb, k0] (fp32 data on stage 0, bf16 activation otherwise).
        Returns the stage output activation (bf16 [mb, 512]) or None (last stage:
        the logits stay in the kernel's accumulator)."""
        assert x.is_contiguous() and x.shape == (self.mb, self.k0)
        assert x.dtype == (torch.float32 if self.k0 == 784 else torch.bfloat16)
        Lb, s = _lib.lib(), _lib.stream_ptr()
        for l in range(self.nh):
            src = x if l == 0 else self.Hs[i][l - 1]
            key = src.data_ptr()
            if self._fwd[i][l] is None or self._keys[i][l] != key:
                self._fwd[i][l] = self._base(i, l, key)
                self._keys[i][l] = key
            head = int(self.last and l == self.nh - 1)
            _lib.check(Lb.jdt_md_layer(ctypes.byref(self._fwd[i][l]), 0, head, s), "md_fwd(stage)")
        return None if self.last else self.Hs[i][self.nh - 1]

    def backward(self, i: int, labels: Optional[torch.Tensor] = None, dh: Optional[torch.Tensor] = None,
                 need_dx: bool = False) -> Optional[torch.Tensor]:
        """Microbatch i, after its forward: CE from ``labels`` (last stage) or the
        output gradient ``dh`` (bf16 [mb, 512]) from the next stage; grads += ;
        returns dX (bf16 [mb, k0]) for the previous stage if ``need_dx``."""
        Lb, s = _lib.lib(), _lib.stream_ptr()
        dZ = self.dZs[i % self.n_sets]
        for l in reversed(range(self.nh)):
            top = l == self.nh - 1
            a = self._bwd[i][l]
            if a is None:
                a = self._base(i, l, 0)
                if l >= 1 or need_dx:
                    a.dZout = dZ[l].data_ptr()
                if not top:
                    a.dZn = dZ[l + 1].data_ptr()
                    a.Wn0 = a.Wn1 = self.P.s(self.kn[l + 1]).data_ptr()
                self._bwd[i][l] = a
            if top and self.last:
                assert labels is not None and labels.dtype == torch.int32 and labels.is_contiguous()
                a.labels = labels.data_ptr()
                variant = 1
            elif top:
                assert dh is not None and dh.dtype == torch.bfloat16 and dh.is_contiguous()
                a.dH = dh.data_ptr()
                variant = 2
            else:
                variant = 0
            _lib.check(Lb.jdt_md_layer(ctypes.byref(a), 1, variant, s), "md_bwd(stage)")
        if not need_dx:
            return None
        K.gemm(dZ[0], self.P.s(self.kn[0]), a_layout="mk", b_layout="nk", out=self.dX[i])
        return self.dX[i]
