"""FusedAdam: torch.optim.Adam semantics (models/model.py:121-122: Adam(lr=2e-4,
betas=(0.5, 0.999))) as one multi-tensor HIP kernel per step (fg_adam_step).

State dict layout is identical to torch.optim.Adam ('step' as a CPU float32 tensor,
'exp_avg', 'exp_avg_sq'; same param_group keys), so checkpoints written by the reference's
Model.save_results (models/model.py:335-355) load into it and vice versa.
"""
import torch

from . import ops


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0, amsgrad=False, *,
                 foreach=None, maximize=False, capturable=False, differentiable=False, fused=None,
                 decoupled_weight_decay=False):
        if weight_decay != 0 or amsgrad or maximize or capturable or differentiable or decoupled_weight_decay:
            raise NotImplementedError("FusedAdam implements the reference's configuration only "
                                      "(weight_decay=0, amsgrad/maximize/capturable/differentiable off)")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad, maximize=maximize,
                        foreach=foreach, capturable=capturable, differentiable=differentiable, fused=fused,
                        decoupled_weight_decay=decoupled_weight_decay)
        super().__init__(params, defaults)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            beta1, beta2 = group["betas"]
            by_step = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                if not p.is_contiguous() or not p.grad.is_contiguous():
                    raise RuntimeError("FusedAdam needs contiguous parameters and gradients")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                by_step.setdefault(int(st["step"].item()), []).append(
                    (p, p.grad, st["exp_avg"], st["exp_avg_sq"]))
            for step, entries in by_step.items():
                ops.adam_step(entries, group["lr"], beta1, beta2, group["eps"], step)
        return loss
