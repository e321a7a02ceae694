"""Losses — same API as src/atmonr/losses.py:5-33, computed by the K9 kernel.

Each ``*_loss(pred, gt, max_i)`` returns the scalar loss and back-propagates into
``pred`` with the reference's gradient. :func:`indexed_loss` is the fused form used by
the pipelines: it gathers ``take_along_dim(color_map, irgb_idx)`` (instant_ngp.py:259-263)
inside the kernel and writes dL/dcolor_map directly.
"""

from __future__ import annotations

import torch

from . import _lib
from ._lib import LOSS_CODES, call, dtype_code, ptr


class _IndexedLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, color_map, irgb_idx, gt, max_i: float, code: int):
        B, C = color_map.shape
        dev = color_map.device
        cm = color_map.contiguous()
        idx = irgb_idx.to(torch.int64).contiguous()
        g = gt.float().contiguous()
        loss = torch.empty((), device=dev, dtype=torch.float32)
        grad = torch.empty_like(cm) if ctx.needs_input_grad[0] else None
        ws = torch.empty(int(_lib.load().anr_loss_workspace_bytes(B)) // 4 + 1, device=dev)
        call("anr_loss_fwd_bwd", code, ptr(cm), dtype_code(cm.dtype), C, ptr(idx), ptr(g), B,
             float(max_i), 1.0, ptr(loss), ptr(grad), ptr(ws), _lib.stream(dev))
        ctx.save_for_backward(grad)
        return loss.to(color_map.dtype)

    @staticmethod
    def backward(ctx, dloss):
        (grad,) = ctx.saved_tensors
        if grad is None:
            return None, None, None, None, None
        return (grad * dloss.to(grad.dtype)), None, None, None, None


class _IndexedLossRef16Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, color_map, irgb_idx, gt, max_i: float, code: int):
        B, C = color_map.shape
        dev = color_map.device
        cm = color_map.to(torch.float16).contiguous()
        idx = irgb_idx.to(torch.int64).contiguous()
        g = gt.float().contiguous()
        loss = torch.empty((), device=dev, dtype=torch.float32)
        grad = torch.empty_like(cm) if ctx.needs_input_grad[0] else None
        ws = torch.empty(int(_lib.load().anr_loss_workspace_bytes(B)) // 4 + 1, device=dev)
        call("anr_loss_ref16_fwd_bwd", code, ptr(cm), C, ptr(idx), ptr(g), B, float(max_i),
             ptr(loss), ptr(grad), ptr(ws), _lib.stream(dev), tag="loss")
        ctx.save_for_backward(grad)
        return loss.to(torch.float16)

    @staticmethod
    def backward(ctx, dloss):
        (grad,) = ctx.saved_tensors
        if grad is None:
            return None, None, None, None, None
        return (grad * dloss.to(grad.dtype)), None, None, None, None


def indexed_loss_ref16(name: str, color_map: torch.Tensor, irgb_idx: torch.Tensor,
                       gt: torch.Tensor, max_i: float) -> torch.Tensor:
    """:func:`indexed_loss` with the reference's f16 numerics (instant_ngp.py:259-263 on
    an f16 colour map: the target cast to f16, every loss op and its autograd in f16;
    csrc/ref16.hip, restated in oracle/ref_f16.py). Returns an f16 scalar."""
    return _IndexedLossRef16Fn.apply(color_map, irgb_idx, gt, float(max_i),
                                     LOSS_CODES[name.lower()])


def indexed_loss(name: str, color_map: torch.Tensor, irgb_idx: torch.Tensor, gt: torch.Tensor,
                 max_i: float) -> torch.Tensor:
    """loss_fn(take_along_dim(color_map, irgb_idx[:, None], 1)[:, 0], gt, max_i)."""
    return _IndexedLossFn.apply(color_map, irgb_idx, gt, float(max_i), LOSS_CODES[name.lower()])


def _flat(name, pred, gt, max_i):
    zeros = torch.zeros(pred.shape[0], dtype=torch.int64, device=pred.device)
    return _IndexedLossFn.apply(pred.reshape(-1, 1), zeros, gt.reshape(-1), float(max_i),
                                LOSS_CODES[name])


def dark_loss(pred, gt, max_i):
    return _flat("dark", pred, gt, max_i)


def hdr_loss(pred, gt, max_i):
    return _flat("hdr", pred, gt, max_i)


def l1_loss(pred, gt, max_i):
    return _flat("l1", pred, gt, max_i)


def l1_plus_hdr_loss(pred, gt, max_i):
    return _flat("l1_plus_hdr", pred, gt, max_i)


def mse_loss(pred, gt, max_i):
    return _flat("mse", pred, gt, max_i)


def mse_plus_hdr_loss(pred, gt, max_i):
    return _flat("mse_plus_hdr", pred, gt, max_i)


LOSSES = {
    "dark": dark_loss,
    "hdr": hdr_loss,
    "l1": l1_loss,
    "l1_plus_hdr": l1_plus_hdr_loss,
    "mse": mse_loss,
    "mse_plus_hdr": mse_plus_hdr_loss,
}
