"""Adam whose update runs in libkge_hip.so (kge_adam_update): the optimizer of the reference's train
step (supervisor.py:26 `optimizer.apply_gradients`; run.py:111 `tf.keras.optimizers.Adam`).

semantics="keras" (default, the TF reference): eps=1e-7 added to sqrt(v), bias correction folded
into the step size; semantics="torch": torch.optim.Adam's update (eps added to sqrt(v_hat)).
"""
from __future__ import annotations

import torch

from . import _lib
from ._lib import check


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
            lr = group["lr"]() if callable(group["lr"]) else group["lr"]
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
                st["step"] += 1
                rc = lib.kge_adam_update(p.data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(),
                                         st["exp_avg_sq"].data_ptr(), p.numel(), float(lr), float(b1),
                                         float(b2), float(group["eps"]), int(st["step"]),
                                         int(group["semantics"] == "keras"), 0,
                                         torch.cuda.current_stream(p.device).cuda_stream)
                check(rc, "kge_adam_update")
        return loss
