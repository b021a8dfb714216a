"""Fused Adam over the flat arena.

A drop-in ``torch.optim.Optimizer`` (so ``LambdaLR`` / ``ReduceLROnPlateau``
drive it through ``param_groups[0]["lr"]``) whose ``step()`` is ONE HIP launch
over every parameter (``pbx_adam_flat``).  Its ``state_dict()`` has exactly
the format of ``torch.optim.Adam`` so reference-style checkpoints
(``optimizer_state_dict``, ``ProteinBERT/utils.py:327-335``) load either way.
"""
from __future__ import annotations

import math
from typing import Any, Dict, Optional

import torch

from .arena import FlatArena


def _hip_ok(t: torch.Tensor) -> bool:
    if t.device.type != "cuda":
        return False
    from ..ops import _lib
    if not _lib.available():
        raise _lib.HipError("GPU run but the HIP kernel library is not built; run ops.build")
    return True


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 0.0, arena: Optional[FlatArena] = None, bf16_shadow: Optional[bool] = None):
        if isinstance(params, FlatArena):
            arena, params = params, params.params
        params = [p for p in params if p.requires_grad]
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, amsgrad=False,
                        maximize=False, foreach=None, capturable=False, differentiable=False, fused=None,
                        decoupled_weight_decay=False)
        super().__init__(params, defaults)
        if len(self.param_groups) != 1:
            raise ValueError("FusedAdam supports one param group (the flat arena)")
        self.arena = arena if arena is not None else FlatArena(self.param_groups[0]["params"])
        a = self.arena
        self.exp_avg = torch.zeros_like(a.data)
        self.exp_avg_sq = torch.zeros_like(a.data)
        if bf16_shadow is None:   # default: keep a bf16 weight mirror whenever the arena is on the GPU
            bf16_shadow = a.data.is_cuda
        self.shadow = a.data.to(torch.bfloat16) if bf16_shadow else None
        if self.shadow is not None:
            a.attach_bf16_shadow(self.shadow)
        self.step_count = 0
        self.grad_scale = 1.0   # set to 1/world by the DP wrapper (SUM all-reduce -> mean)
        self.skip_flag: Optional[torch.Tensor] = None  # device int32; non-zero -> skip update
        dev = a.data.device
        # device-resident hyper-parameters + step counter: the update launch reads everything from
        # device memory, so it can be captured in a hipGraph and replayed; the host only rewrites
        # the hyper-parameter block when lr/betas/... change (prepare(), never during capture)
        self._hp_dev = torch.zeros(8, dtype=torch.float32, device=dev)
        self._step_dev = torch.zeros(1, dtype=torch.float32, device=dev)
        self._hp_host = None
        self._index = {id(p): a.param_index()[id(p)] for p in self.param_groups[0]["params"]}

    # ---------------------------------------------------------------------------------
    def zero_grad(self, set_to_none: bool = False) -> None:  # noqa: ARG002 - arena grads are views
        self.arena.zero_grad()

    def _hparam_values(self):
        g = self.param_groups[0]
        b1, b2 = g["betas"]
        t = max(1, self.step_count)
        return (float(g["lr"]), float(b1), float(b2), float(g["eps"]), float(g["weight_decay"]),
                1.0 - b1 ** t, math.sqrt(1.0 - b2 ** t), float(self.grad_scale))

    def prepare(self) -> None:
        """Push changed hyper-parameters (lr from a scheduler, grad scale) to the device block.
        Host -> device copy: call outside graph capture (the captured step reads the block)."""
        vals = self._hparam_values()
        key = vals[:5] + vals[7:]
        if key != self._hp_host:
            self._hp_dev.copy_(torch.tensor(vals, dtype=torch.float32))
            self._hp_host = key

    def sync_step_counter(self) -> None:
        self._step_dev.fill_(float(self.step_count))

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        self.begin_step()
        self.step_range(0, self.arena.numel)
        return loss

    @torch.no_grad()
    def begin_step(self) -> None:
        """Advance the step counters once per optimizer step; the update itself is one or more
        :meth:`step_range` launches (the DP path updates gradient buckets as their all-reduce lands)."""
        self.step_count += 1
        a = self.arena
        if not a.grads_attached():
            a.attach_grads()
        if _hip_ok(a.data):
            if not torch.cuda.is_current_stream_capturing():
                self.prepare()
            from ..ops import _lib
            _lib.call("pbx_add_scalar", self._step_dev.data_ptr(), 1.0, _lib.stream_ptr(self._step_dev.device))

    @torch.no_grad()
    def step_range(self, start: int, end: int) -> None:
        """Adam on arena elements ``[start, end)`` (element-wise, so any split of the arena gives the
        bitwise result of one whole-arena launch); ``start`` is a segment boundary (16-B aligned)."""
        a = self.arena
        if end <= start:
            return
        if _hip_ok(a.data):
            from ..ops import _lib
            f4, b2 = 4 * start, 2 * start
            _lib.call("pbx_adam_flat", a.data.data_ptr() + f4, a.grad.data_ptr() + f4, self.exp_avg.data_ptr() + f4,
                      self.exp_avg_sq.data_ptr() + f4, None if self.shadow is None else self.shadow.data_ptr() + b2,
                      end - start, self._hp_dev.data_ptr(), _lib.ptr(self.skip_flag), self._step_dev.data_ptr(),
                      _lib.stream_ptr(a.data.device))
        else:
            if skip_requested(self.skip_flag):
                return
            sl = slice(start, end)
            adam_update_host(self, a.data[sl], a.grad[sl], self.exp_avg[sl], self.exp_avg_sq[sl])
            if self.shadow is not None:
                self.shadow[sl].copy_(a.data[sl])

    @torch.no_grad()
    def set_nonfinite_skip(self) -> torch.Tensor:
        """Device flag (int32 [1]): 1 when any arena gradient is NaN / Inf; the update then leaves
        parameters and moments unchanged.  No host sync (two HIP launches on a GPU)."""
        a = self.arena
        if _hip_ok(a.grad):
            from ..ops import _lib
            if getattr(self, "_nf_ws", None) is None:
                self._nf_ws = torch.empty(1025, dtype=torch.int32, device=a.grad.device)
            _lib.call("pbx_nonfinite_flag", a.grad.data_ptr(), a.numel, self._nf_ws.data_ptr(),
                      self._nf_ws[1024:].data_ptr(), float("inf"), 0, _lib.stream_ptr(a.grad.device))
            self.skip_flag = self._nf_ws[1024:]
        else:
            # exact per-element test in one BLAS pass: grad . 0 is NaN iff some element is NaN / Inf (every
            # finite product is exactly 0, so large finite gradients cannot overflow it, unlike a sum)
            z = getattr(self, "_zero_vec", None)
            if z is None or z.numel() != a.grad.numel() or z.dtype != a.grad.dtype:
                z = self._zero_vec = torch.zeros_like(a.grad)
            bad = not bool(torch.isfinite(torch.dot(a.grad, z)))
            self.skip_flag = torch.tensor([1 if bad else 0], dtype=torch.int32)
        return self.skip_flag

    @torch.no_grad()
    def clip_grad_norm_(self, max_norm: float) -> torch.Tensor:
        """Global L2 grad-norm clip over the arena (after DP reduction); returns the pre-clip norm."""
        a = self.arena
        if _hip_ok(a.grad):
            from ..ops import _lib
            ws = torch.empty(1025, dtype=torch.float32, device=a.grad.device)
            _lib.call("pbx_sumsq_flat", a.grad.data_ptr(), a.numel, ws.data_ptr(), ws[1024:].data_ptr(),
                      _lib.stream_ptr(a.grad.device))
            # sumsq of the (grad_scale-scaled) mean gradient: the clip coefficient max_norm / norm
            # is scale-invariant once both sides refer to the same gradient, so the raw threshold
            # is passed (the coefficient multiplies the unscaled SUM gradient in place)
            sumsq = ws[1024:] * (self.grad_scale ** 2)
            _lib.call("pbx_clip_scale_flat", a.grad.data_ptr(), a.numel, sumsq.data_ptr(),
                      float(max_norm), _lib.stream_ptr(a.grad.device))
            return sumsq.sqrt()[0]
        norm = (a.grad * self.grad_scale).norm()
        c = max_norm / (norm + 1e-6)
        if c < 1:
            a.grad.mul_(c)
        return norm

    # ---------------------------------------------------------------------------------
    def state_dict(self) -> Dict[str, Any]:
        g = self.param_groups[0]
        state = {}
        if self.step_count > 0:
            for i, p in enumerate(g["params"]):
                o, n = self.arena.segment(self._index[id(p)])
                state[i] = {"step": torch.tensor(float(self.step_count)),
                            "exp_avg": self.exp_avg[o:o + n].view(p.shape).clone(),
                            "exp_avg_sq": self.exp_avg_sq[o:o + n].view(p.shape).clone()}
        group = {k: v for k, v in g.items() if k != "params"}
        group["params"] = list(range(len(g["params"])))
        return {"state": state, "param_groups": [group]}

    @torch.no_grad()
    def load_state_dict(self, state_dict: Dict[str, Any]) -> None:
        g = self.param_groups[0]
        groups = state_dict["param_groups"]
        if len(groups) != 1 or len(groups[0]["params"]) != len(g["params"]):
            raise ValueError("optimizer state does not match the parameter list")
        for k, v in groups[0].items():
            if k != "params":
                g[k] = tuple(v) if k == "betas" else v
        st = state_dict["state"]
        steps = 0
        for i, p in enumerate(g["params"]):
            if i not in st and str(i) not in st:
                continue
            s = st[i] if i in st else st[str(i)]
            o, n = self.arena.segment(self._index[id(p)])
            self.exp_avg[o:o + n].copy_(s["exp_avg"].reshape(-1))
            self.exp_avg_sq[o:o + n].copy_(s["exp_avg_sq"].reshape(-1))
            steps = int(float(s["step"]))
        self.step_count = steps
        self.sync_step_counter()


def skip_requested(flag: Optional[torch.Tensor]) -> bool:
    return flag is not None and bool(flag.reshape(-1)[0].item())


def adam_update_host(opt: FusedAdam, p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor) -> None:
    """In-place Adam on flat host tensors with ``opt``'s hyper-parameters (torch's fused CPU kernel)."""
    lr, b1, b2, eps, wd, _, _, gs = opt._hparam_values()
    grad = g if gs == 1.0 else g * gs
    if getattr(opt, "_host_step", None) is None:
        opt._host_step = torch.zeros((), dtype=torch.float32)
    opt._host_step.fill_(float(max(1, opt.step_count)))
    torch._fused_adam_([p], [grad], [m], [v], [], [opt._host_step], amsgrad=False, lr=lr, beta1=b1, beta2=b2,
                       weight_decay=wd, eps=eps, maximize=False)


def make_optimizer(model: torch.nn.Module, lr: float = 2e-4, betas=(0.9, 0.999), eps: float = 1e-8,
                   weight_decay: float = 0.0, arena: Optional[FlatArena] = None) -> FusedAdam:
    return FusedAdam(model.parameters() if arena is None else arena.params, lr=lr, betas=betas, eps=eps,
                     weight_decay=weight_decay, arena=arena)
