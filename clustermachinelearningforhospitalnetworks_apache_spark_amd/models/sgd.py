"""Data-parallel mini-batch SGD for binomial logistic regression (BASELINE config 4: "DP SGD with
RCCL grad all-reduce").

One step = one K13 pass over this rank's next ``batch`` rows (the kernel reads the batch position
from a device scalar), the K13b fixed-order sum of its per-block partials into the [d+3] message,
an all-reduce of that message, and the K14 momentum update on the device (which also advances
the batch position and writes the scaled coefficients the next K13 reads) — 3 kernels, no host
synchronisation. On a single rank the step is captured once as a HIP graph and replayed; with
several ranks it runs eagerly (the RCCL all-reduce is not captured).
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from ..ops import glm_ops


class LogisticSGD:
    def __init__(self, x: torch.Tensor, d: int, y: torch.Tensor, weight: Optional[torch.Tensor], comm, batch: int,
                 lr: float, momentum: float, l2: float = 0.0, fit_intercept: bool = True,
                 scale: Optional[torch.Tensor] = None, use_graph: Optional[bool] = None):
        self.x, self.d, self.comm = x, d, comm
        dev = x.device
        self.n = int(x.shape[0])
        self.batch = max(1, min(int(batch), max(self.n, 1)))
        self.nb = max(1, self.n // self.batch)
        self.y = y.to(device=dev, dtype=torch.float64).contiguous()
        self.w = None if weight is None else weight.to(device=dev, dtype=torch.float64).contiguous()
        self.l2, self.fi, self.mom = float(l2), bool(fit_intercept), float(momentum)
        self.coef = torch.zeros(d + 1, dtype=torch.float64, device=dev)
        self.vel = torch.zeros_like(self.coef)
        self.lr = torch.full((), float(lr), dtype=torch.float64, device=dev)
        self.loss_acc = torch.zeros((), dtype=torch.float64, device=dev)
        self.base = torch.zeros((), dtype=torch.int64, device=dev)
        one = torch.ones(1, dtype=torch.float64, device=dev)
        self.kscale = None if scale is None else torch.cat([scale.to(dev, torch.float64), one])
        self.gscale = self.kscale
        self.eff = self.coef.clone()  # coef ⊙ kscale: what K13 reads (kept current by K14)
        self.steps = 0
        if use_graph is None:
            use_graph = x.is_cuda and comm.world_size == 1 and self.n >= self.batch
        self.use_graph = bool(use_graph)
        self._graph = None

    # ------------------------------------------------------------------ one step
    def _body(self):
        msg = glm_ops.logreg_grad(self.x, self.d, self.y, self.eff, self.w, batch=self.batch, row_base=self.base)
        self.comm.allreduce_(msg)
        glm_ops.sgd_update(msg, self.d, self.coef, self.vel, self.eff, self.lr, self.mom, self.l2, self.fi,
                           self.gscale, self.kscale, self.loss_acc, self.base, self.batch, self.nb * self.batch)

    def step(self) -> None:
        if self.use_graph:
            if self._graph is None:
                # warm-up run (lazy allocations, kernel loading) on saved state, then capture
                state = (self.coef, self.vel, self.eff, self.loss_acc, self.base)
                saved = [t.clone() for t in state]
                self._body()
                for t, s in zip(state, saved):
                    t.copy_(s)
                torch.cuda.synchronize(self.x.device)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    self._body()
                self._graph = g
            self._graph.replay()
        else:
            self._body()
        self.steps += 1

    def set_lr(self, lr: float) -> None:
        self.lr.fill_(float(lr))

    def epoch(self, epoch_index: int, lr0: float, steps: Optional[int] = None) -> float:
        """One pass (default nb steps; SPMD callers pass the global max) at lr0/sqrt(1+epoch);
        returns the mean mini-batch loss."""
        steps = self.nb if steps is None else steps
        self.set_lr(lr0 / math.sqrt(1.0 + epoch_index))
        self.loss_acc.zero_()
        for _ in range(steps):
            self.step()
        return float(self.loss_acc.item()) / max(steps, 1)
