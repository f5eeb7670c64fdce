"""Branch replay for numerics oracles: the discrete forward decisions of one run (ReLU
masks, max-pool argmax) recorded and replayed into another run of the same program.

A pre-activation within ~1e-7 of zero flips its ReLU mask under fp32 rounding and moves that
element's gradient by O(1); at random init a training step has many such near-ties, and
which side an fp32 computation lands on is decided by rounding (torch-fp32 itself lands on
the other side of fp64 on some steps).  An fp64 oracle that replays the device run's
branches measures the arithmetic error alone (tests/test_gpu_f32.py, tools/smoke.py)."""
from __future__ import annotations

import torch


class BranchReplay:
    """Records ``bn_train`` / ``conv2d`` ReLU masks and ``maxpool2d`` indices of one run
    (``wrap(module)`` overrides, ``replay = False``) and imposes them on the next
    (``replay = True``).  Only valid images (``nval``) are replayed."""

    def __init__(self, nval):
        self.nval, self.rec, self.replay, self.i = nval, [], False, 0

    def wrap(self, mod):
        o_bn, o_conv, o_mp = mod.bn_train, mod.conv2d, mod.maxpool2d

        def bn_train(y, gamma, beta, rmean, rvar, nvalid, momentum, eps, relu, residual):
            out, m, s = o_bn(y, gamma, beta, rmean, rvar, nvalid, momentum, eps, relu, residual)
            return (self._relu(out) if relu else out), m, s

        def conv2d(*a, **k):
            y = o_conv(*a, **k)
            return self._relu(y) if k.get("relu", a[7] if len(a) > 7 else False) else y

        def maxpool2d(x, kk, st, p):
            y, ind = o_mp(x, kk, st, p)
            return self._pool(x, y, ind)
        return {"bn_train": bn_train, "conv2d": conv2d, "maxpool2d": maxpool2d}

    def _valid(self, t):
        v = torch.zeros(t.shape[:2], dtype=torch.bool)
        for g in range(t.shape[0]):
            v[g, :int(self.nval[g])] = True
        return v.view(*t.shape[:2], *([1] * (t.dim() - 2))).to(t.device)

    def _relu(self, out):
        if not self.replay:
            self.rec.append((out > 0).cpu())
            return out
        m = self.rec[self.i].to(out.device) & self._valid(out)
        self.i += 1
        pos = out > 0
        keep = self._valid(out)
        out = torch.where(keep & m & ~pos, torch.full_like(out, 1e-300), out)
        return torch.where(keep & ~m & pos, torch.zeros_like(out), out)

    def _pool(self, x, y, ind):
        if not self.replay:
            self.rec.append(ind.cpu())
            return y, ind
        hind = torch.where(self._valid(ind).cpu(), self.rec[self.i], ind.cpu()).to(ind.device)
        self.i += 1
        G, N, Hh, Ww, C = x.shape
        yy = x.reshape(G, N, Hh * Ww, C).gather(2, hind.reshape(G, N, -1, C).long()).reshape(y.shape)
        return yy.to(y.dtype), hind.to(ind.dtype)
