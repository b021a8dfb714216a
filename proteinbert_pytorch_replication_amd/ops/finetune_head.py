"""Per-residue fine-tuning head on MI355X (BASELINE cfg 5).

``logits = h Wᵀ + b`` over ``[B*L, 128]`` bf16 encoder rows and K <= 16 classes.  The head weight
stays an fp32 parameter and the logits keep fp32 accuracy: one streaming kernel (``csrc/finetune.hip``
``token_head_fwd``, a thread per residue, W broadcast from LDS) runs fp32 FMAs over the exact bf16
rows -- the fp32 ``F.linear`` result on an upcast copy, memory-bound on the 67 MB row read at
B*L = 262,144 (round 3-4 used two library bf16 GEMMs on a hi / lo weight split, 2 x 25 us).  The weight gradient, a 262,144-long reduction that hipBLASLt ran at 230-410 us,
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
_lib.register("pbx_token_head_fwd", [_P, _P, _P, _P, _L, _I, _P])


def supported(h: torch.Tensor, n_classes: int) -> bool:
    return h.is_cuda and h.dtype == torch.bfloat16 and h.shape[-1] == 128 and n_classes <= 16


class TokenHeadFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, weight, bias):
        B, L, C = h.shape
        h2 = h.contiguous().view(B * L, C)
        K = weight.shape[0]
        # one streaming pass: fp32 FMAs over the exact bf16 rows and fp32 weights (csrc/finetune.hip)
        logits = torch.empty((B * L, K), dtype=torch.float32, device=h.device)
        _lib.call("pbx_token_head_fwd", h2.data_ptr(), weight.detach().float().contiguous().data_ptr(),
                  bias.detach().float().contiguous().data_ptr(), logits.data_ptr(), B * L, K,
                  _lib.stream_ptr(h.device))
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
