"""Fused optimizers over flat buffers: ``FusedSGD``, ``FusedAdam``, ``FusedAdamW``.

Drop-in ``torch.optim.Optimizer`` subclasses for code that does not go through the consensus
engine. At construction every parameter of a param group becomes a view into
ONE flat buffer per (group, device, dtype), and its ``.grad`` a view into a matching flat
gradient buffer (same shape and strides, so channels_last weights stay channels_last), so
autograd accumulates straight into the flat gradient. ``step()`` is then ONE launch of the fused
aggregation + update kernel per flat buffer (``csrc/kernels/agg_update.hip`` with n = 1 worker:
the "aggregate" is the gradient itself), instead of a kernel chain per parameter:

  * SGD: weight decay, momentum (first step: buffer <- g, as torch.optim.SGD), Nesterov
  * Adam: L2 weight decay added to the gradient (torch.optim.Adam); AdamW: decoupled decay
  * bf16 / fp16 parameters keep an fp32 master copy in the optimizer and are rewritten from it
    in the same pass; fp32 parameters are updated in place
  * ``grad_scale``: gradients are multiplied by it inside the kernel (AMP un-scaling)

State is exposed the torch.optim way: ``self.state[p]`` holds views into the flat state
buffers under torch's keys (``momentum_buffer`` / ``exp_avg``, ``exp_avg_sq``, ``step``), plus
``master`` for low-precision parameters, so ``state_dict()`` has torch's format and a
``torch.optim.SGD / Adam / AdamW`` state dict loads into the fused optimizer (and back).

Differences from torch.optim: a parameter whose gradient was never produced is still updated
with a zero gradient (weight decay and momentum still act on it); ``zero_grad`` always zeroes
the flat gradient in place (``set_to_none`` is ignored: ``None`` grads would detach the views).
Replacing ``p.data`` after construction (e.g. ``model.to()``) detaches the parameter from the
flat buffer: build the optimizer after moving the model.

CPU tensors run the same update through the fp32 oracle of ``ops.reference`` (tests).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch

from ..ops.kernels import OptArgs, agg_update

ALIGN = 8        # elements: every parameter starts 16-byte aligned in its flat buffer
PAD = 64         # flat length padding (one 128-byte line of bf16)


class _Flat:
    """Flat parameter / gradient / state storage of one (param group, device, dtype)."""

    def __init__(self, params: List[torch.nn.Parameter], n_state: int):
        self.params = params
        dev, dt = params[0].device, params[0].dtype
        self.offsets: List[int] = []
        off = 0
        for p in params:
            self.offsets.append(off)
            off += -(-p.numel() // ALIGN) * ALIGN
        self.total = -(-max(off, 1) // PAD) * PAD
        self.param = torch.zeros(self.total, dtype=dt, device=dev)
        self.grad = torch.zeros(self.total, dtype=dt, device=dev)
        with torch.no_grad():
            for i, p in enumerate(params):
                v = self.view(self.param, i)
                v.copy_(p.detach())
                p.data = v
        self.lowp = dt != torch.float32
        self.master = self.param.float() if self.lowp else self.param
        self.states = [torch.zeros(self.total, dtype=torch.float32, device=dev)
                       for _ in range(n_state)]
        self.bind_grads()

    def view(self, flat: torch.Tensor, i: int) -> torch.Tensor:
        p = self.params[i]
        return torch.as_strided(flat, p.shape, p.stride(), flat.storage_offset() + self.offsets[i])

    def bind_grads(self) -> None:
        for i, p in enumerate(self.params):
            p.grad = self.view(self.grad, i)

    def sync_foreign_grads(self) -> None:
        """Gradients assigned from outside (``p.grad = t``) are copied into the flat buffer."""
        base = self.grad.data_ptr()
        esz = self.grad.element_size()
        for i, p in enumerate(self.params):
            g = p.grad
            if g is not None and g.data_ptr() == base + self.offsets[i] * esz:
                continue
            v = self.view(self.grad, i)
            if g is None:
                v.zero_()
            else:
                v.copy_(g)
            p.grad = v


class _FusedBase(torch.optim.Optimizer):
    _kind = "sgd"
    _state_keys: Tuple[str, ...] = ()

    def __init__(self, params, defaults):
        super().__init__(params, defaults)
        self._flats: List[List[_Flat]] = []
        for group in self.param_groups:
            by: Dict[Tuple[torch.device, torch.dtype], List[torch.nn.Parameter]] = {}
            for p in group["params"]:
                if not p.requires_grad:
                    continue
                if p.dtype not in (torch.float32, torch.bfloat16, torch.float16):
                    raise TypeError(f"fused optimizers take fp32/bf16/fp16 parameters, not {p.dtype}")
                by.setdefault((p.device, p.dtype), []).append(p)
            flats = [_Flat(ps, len(self._state_keys)) for ps in by.values()]
            self._flats.append(flats)
            group.setdefault("step", 0)
            for fl in flats:
                self._bind_state(fl)

    # ------------------------------------------------------------------ state views
    def _bind_state(self, fl: _Flat) -> None:
        for i, p in enumerate(fl.params):
            st = self.state[p]
            for k, buf in zip(self._state_keys, fl.states):
                st[k] = fl.view(buf, i)
            if fl.lowp:
                st["master"] = fl.view(fl.master, i)

    def state_dict(self):
        for group, flats in zip(self.param_groups, self._flats):
            for fl in flats:
                for p in fl.params:
                    self.state[p]["step"] = torch.tensor(float(group["step"]))
        return super().state_dict()

    def load_state_dict(self, state_dict) -> None:
        # the saved tensors as they are (torch's loader casts state to the parameter dtype,
        # which would round fp32 moments of bf16 parameters)
        raw = {}
        for g, sg in zip(self.param_groups, state_dict["param_groups"]):
            for p, pid in zip(g["params"], sg["params"]):
                if pid in state_dict["state"]:
                    raw[p] = state_dict["state"][pid]
        super().load_state_dict(state_dict)
        # torch rebuilt self.state with fresh tensors: copy the saved values into the flat
        # buffers and point the state back at the views
        for group, flats in zip(self.param_groups, self._flats):
            steps, any_state = [], False
            for fl in flats:
                for i, p in enumerate(fl.params):
                    loaded = raw.get(p, {})
                    for k, buf in zip(self._state_keys, fl.states):
                        if torch.is_tensor(loaded.get(k)):
                            fl.view(buf, i).copy_(loaded[k])
                            any_state = True
                    if fl.lowp:
                        m = loaded.get("master")
                        fl.view(fl.master, i).copy_(m if m is not None else p.detach())
                    if "step" in loaded:
                        steps.append(int(float(loaded["step"])))
            if steps:
                group["step"] = max(steps)
            elif "step" not in group:          # a torch.optim.SGD state dict has no step
                group["step"] = 1 if any_state else 0
            for fl in flats:
                self._bind_state(fl)

    # ------------------------------------------------------------------ training API
    @torch.no_grad()
    def zero_grad(self, set_to_none: bool = True) -> None:
        for flats in self._flats:
            for fl in flats:
                fl.grad.zero_()
                fl.bind_grads()

    def _opt_args(self, group, step: int) -> OptArgs:
        raise NotImplementedError

    @torch.no_grad()
    def step(self, closure=None, grad_scale: float = 1.0):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group, flats in zip(self.param_groups, self._flats):
            group["step"] += 1
            o = self._opt_args(group, group["step"])
            o.gscale = grad_scale
            for fl in flats:
                fl.sync_foreign_grads()
                s1 = fl.states[0] if fl.states else None
                s2 = fl.states[1] if len(fl.states) > 1 else None
                agg_update(fl.grad[None], combine="weighted", n=1, opt=o, master=fl.master,
                           s1=s1, s2=s2, param_out=fl.param if fl.lowp else None)
        return loss

    def flat_buffers(self) -> List[_Flat]:
        return [fl for flats in self._flats for fl in flats]


class FusedSGD(_FusedBase):
    """torch.optim.SGD semantics (dampening 0) in one fused kernel per flat buffer."""
    _kind = "sgd"
    _state_keys = ("momentum_buffer",)

    def __init__(self, params, lr: float = 1e-3, momentum: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False):
        if nesterov and momentum <= 0:
            raise ValueError("Nesterov momentum requires a momentum")
        super().__init__(params, dict(lr=lr, momentum=momentum, weight_decay=weight_decay,
                                      nesterov=nesterov))

    def _opt_args(self, group, step):
        return OptArgs(kind="sgd", lr=group["lr"], momentum=group["momentum"],
                       weight_decay=group["weight_decay"], nesterov=group["nesterov"],
                       first=step == 1)


class FusedAdamW(_FusedBase):
    """torch.optim.AdamW (decoupled weight decay) in one fused kernel per flat buffer."""
    _kind = "adamw"
    _state_keys = ("exp_avg", "exp_avg_sq")

    def __init__(self, params, lr: float = 1e-3, betas: Tuple[float, float] = (0.9, 0.999),
                 eps: float = 1e-8, weight_decay: float = 1e-2):
        super().__init__(params, dict(lr=lr, betas=tuple(betas), eps=eps,
                                      weight_decay=weight_decay))

    def _opt_args(self, group, step):
        b1, b2 = group["betas"]
        return OptArgs(kind=self._kind, lr=group["lr"], weight_decay=group["weight_decay"],
                       beta1=b1, beta2=b2, eps=group["eps"], step=step)


class FusedAdam(FusedAdamW):
    """torch.optim.Adam (L2 weight decay added to the gradient)."""
    _kind = "adam"

    def __init__(self, params, lr: float = 1e-3, betas: Tuple[float, float] = (0.9, 0.999),
                 eps: float = 1e-8, weight_decay: float = 0.0):
        super().__init__(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)


def build_optimizer(name: str, params, **kw) -> torch.optim.Optimizer:
    """``OptimConfig.name`` -> fused optimizer (sgd | adam | adamw)."""
    cls = {"sgd": FusedSGD, "adam": FusedAdam, "adamw": FusedAdamW}[name]
    return cls(params, **kw)
