"""Per-residue fine-tuning head on MI355X (BASELINE cfg 5).

``logits = h Wᵀ + b`` over ``[B*L, 128]`` bf16 encoder rows and K <= 16 classes.  The head weight
stays an fp32 parameter and the logits keep fp32 accuracy: W is split into two bf16 terms
``W = W_hi + W_lo`` (``W_lo = bf16(W - W_hi)``, together exact to ~2^-17 relative) and the bf16
encoder output (exact in fp32) meets both in two bf16 GEMMs accumulating in fp32 -- the same
result as the fp32 ``F.linear`` on an upcast copy to ~1e-6 relative, at 2 x 22 us instead of 75 us
at B*L = 262,144.  The weight gradient, a 262,144-long reduction that hipBLASLt ran at 230-410 us,
is the streaming kernel in ``csrc/finetune.hip`` (fp32 accumulation, deterministic slab reduction);
the input gradient (unfrozen encoders only) is fp32.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from . import global_track  # noqa: F401  (registers pbx_colsum_add)

_P, _I, _L = ctypes.c_void_p, ctypes.c_int, ctypes.c_long
_lib.register("pbx_token_head_wgrad", [_P, _P, _P, _L, _I, _I, _P])


def supported(h: torch.Tensor, n_classes: int) -> bool:
    return h.is_cuda and h.dtype == torch.bfloat16 and h.shape[-1] == 128 and n_classes <= 16


class TokenHeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, weight, bias):
        B, L, C = h.shape
        h2 = h.contiguous().view(B * L, C)
        w_hi = weight.detach().to(torch.bfloat16)
        w_lo = (weight.detach() - w_hi.float()).to(torch.bfloat16)
        logits = torch.addmm(bias.float(), h2, w_hi.t(), out_dtype=torch.float32)
        torch.addmm(logits, h2, w_lo.t(), out_dtype=torch.float32, out=logits)
        ctx.save_for_backward(h2, weight)
        ctx.shape = (B, L)
        return logits.view(B, L, -1)

    @staticmethod
    def backward(ctx, dlogits):
        h2, weight = ctx.saved_tensors
        B, L = ctx.shape
        K = weight.shape[0]
        g = dlogits.reshape(B * L, K).float().contiguous()
        dh = dw = db = None
        if ctx.needs_input_grad[0]:
            dh = torch.mm(g, weight.float()).view(B, L, -1).to(h2.dtype)
        if ctx.needs_input_grad[1]:
            M = B * L
            P = max(1, min(2 * torch.cuda.get_device_properties(h2.device).multi_processor_count, (M + 15) // 16))
            slab = torch.empty((P, K, h2.shape[1]), dtype=torch.float32, device=h2.device)
            st = _lib.stream_ptr(h2.device)
            _lib.call("pbx_token_head_wgrad", h2.data_ptr(), g.data_ptr(), slab.data_ptr(), M, K, P, st)
            dw = torch.zeros_like(weight)
            _lib.call("pbx_colsum_add", slab.data_ptr(), P, K * h2.shape[1], dw.data_ptr(), None, st)
        if ctx.needs_input_grad[2]:
            db = g.sum(dim=0)
        return dh, dw, db
