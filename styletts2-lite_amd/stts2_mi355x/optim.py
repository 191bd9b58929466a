"""Optimizers of the training step (optimizers.py:11-73) with the update on the device as one HIP kernel
per 32 tensors (stts_adamw_step, include/stts2_train.h).

* `AdamW(params, lr, betas, eps, weight_decay)`: torch.optim.AdamW's arithmetic (single-tensor order, amsgrad
  off, decoupled weight decay) and its state layout (`step`, `exp_avg`, `exp_avg_sq` per parameter), so
  `state_dict()` / `load_state_dict()` interoperate with torch.optim.AdamW checkpoints.
* `MultiOptimizer`, `define_scheduler`, `build_optimizer`: the reference's wrappers (optimizers.py:11-73),
  building this AdamW with betas (0.0, 0.99), eps 1e-9, weight decay 1e-4 and OneCycleLR schedulers.
"""
from __future__ import annotations

import ctypes
import weakref
from functools import reduce

import torch
from torch.autograd.graph import increment_version

from .engine import _require_device, _stream, check
from .training import _tl


class _AdamWTensor(ctypes.Structure):
    _fields_ = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
                ("exp_avg_sq", ctypes.c_void_p), ("n", ctypes.c_longlong)]


class AdamW(torch.optim.Optimizer):
    """torch.optim.AdamW (single-tensor arithmetic, bitwise) on stts_adamw_step.  capturable=True (torch's flag):
    the step count of each parameter group lives on the device (stts_adamw_step_dev), so the step can be recorded in
    a hipGraph and replayed; state["step"] is then brought up to date by sync_steps() (one host sync)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, amsgrad=False,
                 capturable=False):
        if amsgrad:
            raise NotImplementedError("amsgrad (the reference does not use it, optimizers.py:66)")
        if not 0.0 <= lr or not 0.0 <= eps or not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"invalid AdamW hyper-parameters lr={lr} betas={betas} eps={eps}")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False))
        self._step_views = weakref.WeakKeyDictionary()  # step tensor -> numpy view of its memory
        self.capturable = bool(capturable)
        self._dev_state = {}  # capturable: group index -> device fp64 [8] (step count, then the step's scalars)

    def sync_steps(self):
        """capturable: copy each group's device step count into its parameters' state["step"] (host sync)."""
        for gi, st in self._dev_state.items():
            n = float(st[0].item())
            for p in self.param_groups[gi]["params"]:
                if p in self.state and "step" in self.state[p]:
                    self.state[p]["step"] = torch.tensor(n)

    def state_dict(self):
        """torch's layout, with the device step counts folded in first (capturable), so a checkpoint carries the
        real step and a resume gets the right bias correction."""
        if self._dev_state:
            self.sync_steps()
        return super().state_dict()

    def load_state_dict(self, state_dict):
        """torch's loader; then every group's device step count (capturable) is re-seeded IN PLACE from the loaded
        state["step"], so a hipGraph recorded against that count keeps its pointer and replays the loaded step."""
        # (the moments too: torch's loader makes new tensors, while a recorded graph holds the old buffers' pointers;
        # the loaded values are copied into the existing buffers)
        old = {p: {k: st[k] for k in ("exp_avg", "exp_avg_sq") if k in st} for p, st in self.state.items()}
        super().load_state_dict(state_dict)
        with torch.no_grad():
            for p, bufs in old.items():
                st = self.state.get(p)
                for k, buf in bufs.items():
                    if st is not None and k in st and st[k].shape == buf.shape and st[k].device == buf.device:
                        buf.copy_(st[k])
                        st[k] = buf
        views = self.__dict__.get("_step_views")
        if views is not None:
            views.clear()  # (the loaded step tensors are new objects)
        for gi, dev in self._dev_state.items():
            steps = {float(self.state[p]["step"]) for p in self.param_groups[gi]["params"]
                     if p in self.state and "step" in self.state[p]}
            if len(steps) > 1:
                raise ValueError(f"capturable AdamW keeps one step count per group; group {gi} loaded {sorted(steps)}")
            with torch.no_grad():
                dev[0].fill_(steps.pop() if steps else 0.0)

    def _step_capturable(self, gi, group):
        beta1, beta2 = group["betas"]
        items = []
        for p in group["params"]:
            if p.grad is None:
                continue
            if p.dtype != torch.float32 or not p.is_cuda or not p.is_contiguous() or not p.grad.is_contiguous():
                raise RuntimeError("HIP AdamW: contiguous fp32 parameters and gradients on the device")
            st = self.state[p]
            if len(st) == 0:
                st["step"] = torch.tensor(0.0)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            items.append((p, p.grad, st["exp_avg"], st["exp_avg_sq"]))
        if not items:
            return
        dev = self._dev_state.get(gi)
        if dev is None:  # one count per group (every parameter of the group steps together), from the host state
            dev = torch.zeros(8, dtype=torch.float64, device=items[0][0].device)
            dev[0] = float(self.state[items[0][0]]["step"])
            self._dev_state[gi] = dev
        arr = (_AdamWTensor * len(items))()
        for i, (p, g, m, v) in enumerate(items):
            arr[i] = _AdamWTensor(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel())
        check(_tl().stts_adamw_step_dev(arr, len(items), ctypes.c_double(group["lr"]), ctypes.c_double(beta1),
                                        ctypes.c_double(beta2), ctypes.c_double(group["eps"]),
                                        ctypes.c_double(group["weight_decay"]), ctypes.c_void_p(dev.data_ptr()),
                                        _stream()), "stts_adamw_step_dev")
        increment_version([p for p, _, _, _ in items])

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        _require_device()
        if self.capturable:
            for gi, group in enumerate(self.param_groups):
                self._step_capturable(gi, group)
            return loss
        for group in self.param_groups:
            beta1, beta2 = group["betas"]
            # tensors of one group that share a step count go in one call (a freshly added parameter starts at 1)
            batches = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("AdamW does not support sparse gradients")
                if p.dtype != torch.float32 or not p.is_cuda or not p.is_contiguous():
                    raise RuntimeError("HIP AdamW: contiguous fp32 parameters on the device")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                # the step count stays torch.optim's 0-d CPU tensor (state_dict compatibility), advanced through a
                # cached numpy view of its memory: a torch op + .item() per parameter was ~5 us of host time each
                t = st["step"]
                if not t.is_cpu:  # (a checkpoint may carry the step on the device)
                    t = st["step"] = t.detach().to("cpu", torch.float32)
                views = self.__dict__.get("_step_views")
                if views is None:  # (not in Optimizer.__getstate__: a deep-copied / unpickled optimizer rebuilds it)
                    views = self._step_views = weakref.WeakKeyDictionary()
                sn = views.get(t)
                if sn is None:
                    sn = views[t] = t.numpy()
                sn += 1
                g = p.grad if p.grad.is_contiguous() and p.grad.dtype == torch.float32 else \
                    p.grad.float().contiguous()
                batches.setdefault(int(sn), []).append((p, g, st["exp_avg"], st["exp_avg_sq"]))
            for step, items in batches.items():
                arr = (_AdamWTensor * len(items))()
                for i, (p, g, m, v) in enumerate(items):
                    arr[i] = _AdamWTensor(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel())
                check(_tl().stts_adamw_step(arr, len(items), ctypes.c_double(group["lr"]), ctypes.c_double(beta1),
                                            ctypes.c_double(beta2), ctypes.c_double(group["eps"]),
                                            ctypes.c_double(group["weight_decay"]), step, _stream()),
                      "stts_adamw_step")
                # the kernel writes through raw pointers: bump each parameter's version counter as torch's
                # in-place update would, so cached packed weights (engine._Engine.stale) see the new values
                increment_version([p for p, _, _, _ in items])
        return loss


class MultiOptimizer:
    """optimizers.py:11-51."""

    def __init__(self, optimizers={}, schedulers={}):
        self.optimizers = optimizers
        self.schedulers = schedulers
        self.keys = list(optimizers.keys())
        self.param_groups = reduce(lambda x, y: x + y, [v.param_groups for v in self.optimizers.values()])

    def state_dict(self):
        return [(key, self.optimizers[key].state_dict()) for key in self.keys]

    def load_state_dict(self, state_dict):
        for key, val in state_dict:
            try:
                self.optimizers[key].load_state_dict(val)
            except Exception:
                print("Unloaded %s" % key)

    def step(self, key=None, scaler=None):
        keys = [key] if key is not None else self.keys
        for k in keys:
            if scaler is not None:
                scaler.step(self.optimizers[k])
                scaler.update()
            else:
                self.optimizers[k].step()

    def zero_grad(self, key=None):
        if key is not None:
            self.optimizers[key].zero_grad()
        else:
            for k in self.keys:
                self.optimizers[k].zero_grad()

    def scheduler(self, *args, key=None):
        if key is not None:
            self.schedulers[key].step(*args)
        else:
            for k in self.keys:
                self.schedulers[k].step(*args)


def define_scheduler(optimizer, params):
    """optimizers.py:53-63."""
    return torch.optim.lr_scheduler.OneCycleLR(
        optimizer, max_lr=params.get("max_lr", 2e-4), epochs=params.get("epochs", 200),
        steps_per_epoch=params.get("steps_per_epoch", 1000), pct_start=params.get("pct_start", 0.0),
        div_factor=1, final_div_factor=1)


def build_optimizer(parameters_dict, scheduler_params_dict, lr):
    """optimizers.py:65-73 with this module's AdamW."""
    optim = {key: AdamW(params, lr=lr, weight_decay=1e-4, betas=(0.0, 0.99), eps=1e-9)
             for key, params in parameters_dict.items()}
    schedulers = {key: define_scheduler(opt, scheduler_params_dict[key]) for key, opt in optim.items()}
    return MultiOptimizer(optim, schedulers)
