"""AssociationFunction on the GPU — the registry of pairwise box similarities the OCSort family
selects with ``asso_func`` (reference: boxmot/utils/iou.py:14-346).

Same surface as the reference class: ``AssociationFunction(w, h, asso_mode)`` exposes
``asso_func`` (chosen by ``_get_asso_func``, :320-346, unknown modes raise ``ValueError``), the
static ``iou_batch / hmiou_batch / giou_batch / diou_batch / ciou_batch`` and the bound
``centroid_batch`` (normalised by the frame diagonal).  Every call runs ``bx_pairwise_cost``
in libbxassoc.so; there is no CPU path (the library is required, ``_native.load`` raises
without it).  Inputs are [N, >=4] xyxy rows, numpy (copied to the device and back) or float64
CUDA tensors (result stays on the device, on torch's current stream).  The oriented-box modes
(``iou_obb``, ``centroid_obb``) need a rotated-rectangle intersection and are not provided.
"""
from __future__ import annotations

import numpy as np

from . import _native

KINDS = {"iou": 0, "hmiou": 1, "giou": 2, "diou": 3, "ciou": 4, "centroid": 5}


def pairwise_cost(kind: str, bboxes1, bboxes2, w: float = 0.0, h: float = 0.0):
    """``<kind>_batch(bboxes1, bboxes2)`` on the GPU -> [N, M] float64."""
    import torch

    if kind not in KINDS:
        raise ValueError(f"Invalid association mode: {kind}. Choose from {list(KINDS)}")
    L = _native.load()
    on_dev = isinstance(bboxes1, torch.Tensor) and bboxes1.is_cuda
    a = _as_dev(torch, bboxes1)
    b = _as_dev(torch, bboxes2)
    if a.shape[1] < 4 or b.shape[1] < 4:
        raise AssertionError("boxes need at least 4 columns (x1, y1, x2, y2)")
    out = torch.empty((a.shape[0], b.shape[0]), dtype=torch.float64, device=a.device)
    stream = torch.cuda.current_stream(a.device).cuda_stream
    _native.check(L.bx_pairwise_cost(KINDS[kind], a.data_ptr(), a.shape[0], a.stride(0),
                                     b.data_ptr(), b.shape[0], b.stride(0), float(w), float(h),
                                     out.data_ptr(), stream))
    if on_dev:
        return out
    return out.cpu().numpy()


def _as_dev(torch, x):
    if isinstance(x, torch.Tensor):
        t = x.to(device="cuda", dtype=torch.float64)
    else:
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(x, np.float64))).cuda()
    if t.dim() == 1:
        t = t.reshape(-1, 4) if t.numel() else t.reshape(0, 4)
    if t.stride(1) != 1:
        t = t.contiguous()
    return t


class AssociationFunction:
    """utils/iou.py:14-49 — frame size (w, h) for ``centroid``; ``asso_func`` per ``asso_mode``."""

    def __init__(self, w, h, asso_mode: str = "iou"):
        self.w = w
        self.h = h
        self.asso_mode = asso_mode
        self.asso_func = self._get_asso_func(asso_mode)

    @staticmethod
    def iou_batch(bboxes1, bboxes2):
        return pairwise_cost("iou", bboxes1, bboxes2)

    @staticmethod
    def hmiou_batch(bboxes1, bboxes2):
        return pairwise_cost("hmiou", bboxes1, bboxes2)

    @staticmethod
    def giou_batch(bboxes1, bboxes2):
        return pairwise_cost("giou", bboxes1, bboxes2)

    @staticmethod
    def diou_batch(bboxes1, bboxes2):
        return pairwise_cost("diou", bboxes1, bboxes2)

    @staticmethod
    def ciou_batch(bboxes1, bboxes2):
        return pairwise_cost("ciou", bboxes1, bboxes2)

    def centroid_batch(self, bboxes1, bboxes2):
        return pairwise_cost("centroid", bboxes1, bboxes2, self.w, self.h)

    @staticmethod
    def run_asso_func(self, bboxes1, bboxes2):
        return self.asso_func(bboxes1, bboxes2)

    def _get_asso_func(self, asso_mode):
        funcs = {
            "iou": AssociationFunction.iou_batch,
            "hmiou": AssociationFunction.hmiou_batch,
            "giou": AssociationFunction.giou_batch,
            "ciou": AssociationFunction.ciou_batch,
            "diou": AssociationFunction.diou_batch,
            "centroid": self.centroid_batch,
        }
        if asso_mode in ("iou_obb", "centroid_obb"):
            raise NotImplementedError(f"{asso_mode}: oriented boxes are not on the engine")
        if asso_mode not in funcs:
            raise ValueError(f"Invalid association mode: {asso_mode}. Choose from "
                             f"{list(funcs.keys())}")
        return funcs[asso_mode]
