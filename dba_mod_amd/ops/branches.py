"""Branch replay for numerics oracles: the discrete forward decisions of one run (ReLU
masks, max-pool argmax) recorded and replayed into another run of the same program — but
ONLY where the replaying run itself sees a near-tie.

A pre-activation within ~1e-7 of zero flips its ReLU mask under fp32 rounding and moves that
element's gradient by O(1); at random init a training step has many such near-ties, and
which side an fp32 computation lands on is decided by rounding (torch-fp32 itself lands on
the other side of fp64 on some steps).  An fp64 oracle that replays the device run's
branches at those ties measures the arithmetic error alone (tests/test_gpu_f32.py,
tools/smoke.py).

A decision the replaying run takes CLEARLY differently is never imposed: a kernel that
zeroes a clearly positive pre-activation, or a max-pool that picks a clearly smaller
element, still shows up as error.  Ties are judged in the replaying run's own values:

* ReLU: ``|pre| <= tol * rms(pre)`` (per replica; the replay runs the op without its fused
  ReLU to see ``pre``);
* max-pool: ``x[recorded index] >= x[own index] - tol * rms(x)``.

``flips`` counts the replayed decisions, ``hard`` the disagreements outside the tie band
(left as they are); ``elements`` the decisions compared.
"""
from __future__ import annotations

import torch

TIE_TOL = 1e-4


class BranchReplay:
    """Records the ReLU masks of the fused training BN (``conv_bn_stats`` lazy outputs,
    ``bn_apply``) and of ``conv2d`` and the ``maxpool2d`` indices of one run
    (``wrap(module)`` overrides, ``replay = False``) and replays them near ties in every
    later run (``replay = True``; :meth:`start_replay` before each).  Only valid images
    (``nval``) are compared."""

    def __init__(self, nval, tol: float = TIE_TOL):
        self.nval, self.rec, self.replay, self.i = nval, [], False, 0
        self.tol = tol
        self.flips = self.hard = self.elements = 0

    def start_replay(self) -> None:
        self.replay, self.i = True, 0
        self.flips = self.hard = self.elements = 0

    def wrap(self, mod):
        o_conv, o_mp = mod.conv2d, mod.maxpool2d
        o_cbs, o_apply = mod.conv_bn_stats, mod.bn_apply

        def conv_bn_stats(x, w, wsel, stride, pad, nvalid, p, relu):
            # the fused training BN (ops.bnstate): a lazy BN+ReLU output's decisions are taken
            # where its value and its backward mask are formed, from stat.relu_mask
            y, st = o_cbs(x, w, wsel, stride, pad, nvalid, p, relu)
            if relu:
                C = y.shape[-1]
                sh = (y.shape[0],) + (1,) * (y.dim() - 2) + (C,)
                # fp64: the exact sign of y * scale + shift, which is the sign of the kernels'
                # fmaf (a correctly rounded fma never crosses zero); fp32 mul-then-add can
                pre = (y.double() * st.coef[:, 2].reshape(sh).double() + st.coef[:, 3].reshape(sh).double())
                if not self.replay:
                    self.rec.append((pre > 0).cpu())
                else:
                    st.relu_mask = self._decide(pre.to(y.dtype) if y.dtype == torch.float64 else pre)
            return y, st

        def bn_apply(a, residual, relu, nvalid=None):
            if not (relu and self.replay):
                out = o_apply(a, residual, relu, nvalid)
                return self._record(out) if relu else out
            return self._relu(o_apply(a, residual, False, nvalid))

        def conv2d(*a, **k):
            relu = k.get("relu", a[7] if len(a) > 7 else False)
            if not (relu and self.replay):
                y = o_conv(*a, **k)
                return self._record(y) if relu else y
            if len(a) > 7:
                a = a[:7] + (False,) + a[8:]
            else:
                k = dict(k, relu=False)
            return self._relu(o_conv(*a, **k))

        def maxpool2d(x, kk, st, p, want_ind=True):
            y, ind = o_mp(x, kk, st, p)   # the decisions are recorded / replayed either way
            y, ind = self._pool(x, y, ind)
            return y, (ind if want_ind else None)

        def basic_block_ok(x, w1, w2):
            # the fused evaluation BasicBlock keeps its mid activation (and so its ReLU
            # decisions) on chip: recorded and replayed runs both take the two convs, whose
            # decisions this oracle sees (the fused kernel has its own fp64 test)
            return False
        # likewise the fused stem block and the fused downsampling block (its shortcut's sum
        # never leaves the chip): both runs take the separate convs
        return {"conv2d": conv2d, "maxpool2d": maxpool2d, "conv_bn_stats": conv_bn_stats, "bn_apply": bn_apply,
                "basic_block_ok": basic_block_ok, "stem_block_ok": lambda x, w0, w1, w2: False,
                "down_block_ok": lambda a, w2, x2, wsc: False}

    def _valid(self, t):
        v = torch.zeros(t.shape[:2], dtype=torch.bool)
        for g in range(t.shape[0]):
            v[g, :int(self.nval[g])] = True
        return v.view(*t.shape[:2], *([1] * (t.dim() - 2))).to(t.device)

    def _rms(self, t):
        """Per-replica rms over the valid images (the tie scale)."""
        keep = self._valid(t).expand_as(t)
        sq = torch.where(keep, t.double() ** 2, torch.zeros((), dtype=torch.float64, device=t.device))
        n = keep.reshape(t.shape[0], -1).sum(1).clamp(min=1)
        r = (sq.reshape(t.shape[0], -1).sum(1) / n).sqrt()
        return r.view(-1, *([1] * (t.dim() - 1))).to(t.dtype)

    def _record(self, out):
        self.rec.append((out > 0).cpu())
        return out

    def _decide(self, pre):
        """The ReLU decisions of ``pre``: its own, with the recorded one taken at near-ties."""
        m = self.rec[self.i].to(pre.device)
        self.i += 1
        keep = self._valid(pre).expand_as(pre)
        pos = pre > 0
        tie = pre.abs() <= self.tol * self._rms(pre)
        differ = keep & (m != pos)
        take = differ & tie
        self.flips += int(take.sum())
        self.hard += int((differ & ~tie).sum())
        self.elements += int(keep.sum())
        return torch.where(take, m, pos)

    def _relu(self, pre):
        m = self.rec[self.i].to(pre.device)
        self.i += 1
        keep = self._valid(pre).expand_as(pre)
        pos = pre > 0
        tie = pre.abs() <= self.tol * self._rms(pre)
        differ = keep & (m != pos)
        take = differ & tie
        self.flips += int(take.sum())
        self.hard += int((differ & ~tie).sum())
        self.elements += int(keep.sum())
        # replayed positive: an (essentially zero) positive value; replayed zero: zero
        out = torch.where(pos, pre, torch.zeros_like(pre))
        out = torch.where(take & m, torch.full_like(pre, 1e-300 if pre.dtype == torch.float64 else 1e-30), out)
        return torch.where(take & ~m, torch.zeros_like(pre), out)

    def _pool(self, x, y, ind):
        if not self.replay:
            self.rec.append(ind.cpu())
            return y, ind
        rec = self.rec[self.i].to(ind.device).to(ind.dtype)
        self.i += 1
        G, N, Hh, Ww, C = x.shape
        xf = x.reshape(G, N, Hh * Ww, C)
        y_rec = xf.gather(2, rec.reshape(G, N, -1, C).long()).reshape(y.shape)
        keep = self._valid(ind).expand_as(ind)
        differ = keep & (rec != ind)
        tie = y_rec >= y - self.tol * self._rms(x).reshape(G, 1, 1, 1, 1)
        take = differ & tie
        self.flips += int(take.sum())
        self.hard += int((differ & ~tie).sum())
        self.elements += int(keep.sum())
        hind = torch.where(take, rec, ind)
        yy = xf.gather(2, hind.reshape(G, N, -1, C).long()).reshape(y.shape)
        return yy.to(y.dtype), hind
