"""Adam whose update runs in libkge_hip.so (kge_adam_update): the optimizer of the reference's train
step (supervisor.py:26 `optimizer.apply_gradients`; run.py:111 `tf.keras.optimizers.Adam`).

semantics="keras" (default, the TF reference): eps=1e-7 added to sqrt(v), bias correction folded
into the step size; semantics="torch": torch.optim.Adam's update (eps added to sqrt(v_hat)).
"""
from __future__ import annotations

import inspect

import torch

from . import _lib
from ._lib import check


def lrfn(epoch, num_replicas=1):
    """run.py:69-84: linear warm-up over 5 epochs from 1e-5 to 5e-5 * replicas, then 0.8 ** epoch decay
    towards 1e-5 (evaluated in float like the @tf.function)."""
    LR_START, LR_MAX, LR_MIN = 0.00001, 0.00005 * num_replicas, 0.00001
    LR_RAMPUP_EPOCHS, LR_SUSTAIN_EPOCHS, LR_EXP_DECAY = 5.0, 0.0, 0.8
    if float(epoch) < LR_RAMPUP_EPOCHS:
        return (LR_MAX - LR_START) / LR_RAMPUP_EPOCHS * float(epoch) + LR_START
    if float(epoch) < LR_RAMPUP_EPOCHS + LR_SUSTAIN_EPOCHS:
        return LR_MAX
    return (LR_MAX - LR_MIN) * LR_EXP_DECAY ** (float(epoch) - LR_RAMPUP_EPOCHS - LR_SUSTAIN_EPOCHS) + LR_MIN


class LRSchedule:
    """run.py:106-108: `lrfn(epoch=step // steps_per_epoch)` as a Keras LearningRateSchedule; Adam
    calls it with the number of updates already applied (Keras' `optimizer.iterations`)."""

    def __init__(self, steps_per_epoch, num_replicas=1):
        self.steps_per_epoch = int(steps_per_epoch)
        self.num_replicas = int(num_replicas)

    def __call__(self, step):
        return lrfn(int(step) // self.steps_per_epoch, self.num_replicas)


def resolve_lr(lr, iterations):
    """A float, a zero-argument callable, or a schedule called with the prior update count."""
    if not callable(lr):
        return float(lr)
    try:
        n = len(inspect.signature(lr).parameters)
    except (TypeError, ValueError):
        n = 1
    return float(lr(iterations) if n else lr())


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=None, semantics="keras"):
        if semantics not in ("keras", "torch"):
            raise ValueError("semantics must be 'keras' or 'torch'")
        if eps is None:
            eps = 1e-7 if semantics == "keras" else 1e-8
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, semantics=semantics))

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        lib = _lib.load()
        for group in self.param_groups:
            first = next((self.state[q] for q in group["params"] if q.grad is not None and self.state[q]), None)
            lr = resolve_lr(group["lr"], first["step"] if first else 0)
            b1, b2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.device.type != "cuda" or p.dtype != torch.float32 or not p.is_contiguous():
                    raise _lib.KGEHipError("Adam: parameters must be contiguous fp32 on a ROCm device")
                g = p.grad
                if not g.is_contiguous():
                    g = p.grad = g.contiguous()
                st = self.state[p]
                if not st:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                rc = lib.kge_adam_update(p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(),
                                         st["exp_avg_sq"].data_ptr(), p.numel(), float(lr), float(b1),
                                         float(b2), float(group["eps"]), int(st["step"]) + 1,
                                         int(group["semantics"] == "keras"), 0,
                                         torch.cuda.current_stream(p.device).cuda_stream)
                check(rc, "kge_adam_update")
                st["step"] += 1  # committed only once the library accepted the update
        return loss
