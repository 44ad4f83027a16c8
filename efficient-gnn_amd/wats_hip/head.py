"""Fused WATS temperature head.

Reference ``calibration/WATS.py``: ``net = Linear(F,16) - ReLU - Linear(16,1)``
(:101-105); ``forward`` computes ``T = log(exp(net(H)) + 1.1)`` and
``log_softmax(logits / T)`` (:124-130), and ``calib_train`` backpropagates the
NLL through it every epoch (:145-151).  :func:`wats_head` is that whole
expression as two HIP kernels (``csrc/head.hip``): forward, and a backward
giving the logits gradient and the four parameter gradients.  Float64 sums in a
fixed order make the backward deterministic.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import check, ptr
from .laplacian import stream_handle


def _c(t):
    return t.detach().to(torch.float32).contiguous()


class _WATSHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, H, logits, W1, b1, W2, b2):
        dev = logits.device
        H, lg, W1c, b1c, W2c, b2c = (_c(t) for t in (H, logits, W1, b1, W2, b2))
        n, C = lg.shape
        F, hid = H.shape[1], W1c.shape[0]
        out = torch.empty(n, C, dtype=torch.float32, device=dev)
        t_save = torch.empty(max(n, 1), dtype=torch.float32, device=dev)
        with torch.cuda.device(dev):
            check(_lib.load().wg_wats_head_forward(n, F, C, hid, ptr(H), ptr(lg), ptr(W1c), ptr(b1c), ptr(W2c),
                                                   ptr(b2c), ptr(out), ptr(t_save), stream_handle(dev)),
                  "wats_head_forward")
        ctx.save_for_backward(H, lg, W1c, b1c, W2c, b2c, out, t_save)
        return out

    @staticmethod
    def backward(ctx, g):
        H, lg, W1, b1, W2, b2, out, t_save = ctx.saved_tensors
        dev = lg.device
        n, C = lg.shape
        F, hid = H.shape[1], W1.shape[0]
        g = g.to(torch.float32).contiguous()
        need_logits = ctx.needs_input_grad[1]
        glog = torch.empty_like(lg) if need_logits else None
        gW1, gb1 = torch.empty_like(W1), torch.empty_like(b1)
        gW2, gb2 = torch.empty_like(W2), torch.empty_like(b2)
        lib = _lib.load()
        nbytes = ctypes.c_int64(0)
        check(lib.wg_wats_head_workspace(n, F, hid, ctypes.byref(nbytes)), "wats_head_workspace")
        ws = torch.empty(max(1, nbytes.value), dtype=torch.uint8, device=dev)
        with torch.cuda.device(dev):
            check(lib.wg_wats_head_backward(n, F, C, hid, ptr(H), ptr(lg), ptr(W1), ptr(b1), ptr(W2), ptr(b2),
                                            ptr(out), ptr(t_save), ptr(g), ptr(glog), ptr(gW1), ptr(gb1), ptr(gW2),
                                            ptr(gb2), ptr(ws), stream_handle(dev)), "wats_head_backward")
        return None, glog, gW1, gb1, gW2, gb2


def wats_head(H: torch.Tensor, logits: torch.Tensor, net: torch.nn.Sequential) -> torch.Tensor:
    """``log_softmax(logits / log(exp(net(H)) + 1.1))`` (WATS.py:124-130) with
    ``net = Sequential(Linear(F, hid), ReLU(), Linear(hid, 1))``."""
    l1, l2 = net[0], net[2]
    if H.dim() == 1:
        H = H.reshape(-1, 1)
    return _WATSHead.apply(H, logits, l1.weight, l1.bias, l2.weight, l2.bias)
