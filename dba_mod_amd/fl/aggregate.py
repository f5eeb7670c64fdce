"""Server-side aggregation over flat client buffers.

Inputs are the round's client states ``finals [n, S]`` (or summed gradients for FoolsGold),
already gathered onto every rank; each rank applies the identical update redundantly, so no
broadcast is needed and every rank ends the round with a bit-identical global model.

* :func:`fedavg` / :func:`fedavg_apply` — reference ``helper.py:240-257``: ``w += (eta/no_models)
  * sum_i delta_i`` (+ N(0, sigma) per element with ``diff_privacy``); unweighted; applied to
  the BN running stats too (D2).  The delta sum is an fp64 HIP reduction, per rank then
  all-reduced (``Server._aggregate``).  The int64 ``num_batches_tracked`` counters are not part of the float
  bucket (D1: the reference's float→int64 add crashes on modern torch).
* :func:`geometric_median` / :func:`geometric_median_distributed` — RFA / Weiszfeld,
  ``helper.py:295-373`` (the latter with the points resident on their owner ranks): one batched distance
  kernel (all n clients in one pass) and one weighted-sum kernel per iteration; weights and
  the stopping test stay on the device (one host read per aggregation).  Quirk D5 (``wv`` undefined if
  converged at iteration 0) resolves to the current weights.
* The weighted sums of RFA and FoolsGold are REPRODUCIBLE: every product is quantised on its own
  onto a fixed two-limb int64 grid (:func:`fixed_exponent`, ``ops.weighted_sum_fixed``) and the
  limbs are summed exactly — over a rank's clients, then over ranks by an int64 all-reduce — so
  the global model's bits do not depend on the world size or on which rank holds which client.
* :class:`FoolsGold` — ``helper.py:527-607``: cosine similarity of the clients' final-FC
  gradient features (history-summed with ``fg_use_memory``), pardoning, logit weights,
  weighted gradient sum, then one fresh-SGD server step (BN buffers untouched).
"""
from __future__ import annotations

import logging
import math
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import ops

log = logging.getLogger("logger")


def fedavg(global_state: torch.Tensor, finals: torch.Tensor, eta: float, no_models: int,
           dp: bool, sigma: float, seed: int, n_update: int) -> None:
    """In-place FedAvg of ``finals`` [n, S]; ``n_update`` = leading entries aggregated (S or P)."""
    fedavg_apply(global_state, ops.delta_sum(finals[:, :n_update], global_state[:n_update]), eta, no_models,
                 dp, sigma, seed, n_update)


def fedavg_apply(global_state: torch.Tensor, delta_sum: torch.Tensor, eta: float, no_models: int,
                 dp: bool, sigma: float, seed: int, n_update: int) -> None:
    """``w += (eta / no_models) * sum_i delta_i (+ noise)`` from the (all-reduced) fp64 sum of the
    clients' deltas (``ops.delta_sum``: fused HIP kernel on GPU)."""
    ops.add_noise_scaled(global_state[:n_update], delta_sum, eta / no_models, sigma, seed, dp)


FIXED_MAX_TERMS = 512


def fixed_exponent(maxabs: float, n: int) -> Optional[int]:
    """E of the fixed-point weighted sums: with weights <= 1 and |points| <= ``maxabs`` (the max
    over ALL clients, every rank the same), each scaled product |w p 2^E| < 2^52 / n, so neither
    limb sum of n <= 512 products overflows int64.  The grid step is 2^-(E + 53): ~105 bits below
    the largest product.  None when the grid cannot hold the sum — a non-finite ``maxabs`` (a NaN /
    Inf client update: the fp64 sum carries it into the global model, as the reference's torch
    aggregation does, instead of quantising it into finite garbage) or more than 512 terms; the
    callers then take the plain fp64 weighted sum (:func:`wsum_part`)."""
    if n > FIXED_MAX_TERMS or not math.isfinite(maxabs):
        return None
    if not maxabs > 0.0:
        return 0
    n2 = max(0, math.ceil(math.log2(max(1, n))))
    _, ex = math.frexp(maxabs)          # maxabs < 2**ex
    return max(-1000, min(1000, 52 - n2 - ex))


def max_abs(t: Optional[torch.Tensor]) -> float:
    """Host max |t| for :func:`fixed_exponent`, NaN mapped to +inf (so a max-all-reduce over ranks
    sees it whatever the backend does with NaN)."""
    if t is None or t.numel() == 0:
        return 0.0
    v = float(t.abs().max().item())
    return math.inf if math.isnan(v) else v


def wsum_part(points: torch.Tensor, w: torch.Tensor, E: Optional[int]) -> torch.Tensor:
    """A rank's partial of sum_i w_i points_i: [2, L] int64 fixed-point limbs on the 2^E grid
    (exact, order-free), or an fp64 [L] vector when ``E`` is None."""
    if E is None:
        return ops.weighted_sum(points, w.float(), torch.float64)
    return ops.weighted_sum_fixed(points, w.float(), E)


def wsum_zero(L: int, E: Optional[int], device) -> torch.Tensor:
    """The partial of a rank without clients (same shape / dtype as :func:`wsum_part`)."""
    if E is None:
        return torch.zeros(L, dtype=torch.float64, device=device)
    return torch.zeros(2, L, dtype=torch.int64, device=device)


def wsum_decode(part: torch.Tensor, E: Optional[int]) -> torch.Tensor:
    """fp32 value of a (reduced) :func:`wsum_part`."""
    return (part if E is None else fixed_decode(part, E)).float()


def fixed_decode(limbs: torch.Tensor, E: int) -> torch.Tensor:
    """fp64 value of [2, L] int64 limb sums on the 2^-(E + 53) grid (elementwise, exact up to the
    final rounding: the same bits for the same limbs)."""
    return limbs[0].double() * (2.0 ** -E) + limbs[1].double() * (2.0 ** -(E + 53))


def _weiszfeld(avg, dists, alphas: torch.Tensor, maxiter: int, eps: float, ftol: float, poll: int = 0):
    """Weiszfeld iteration control on the DEVICE (reference ``helper.py:320-352``, SURVEY
    §7.4.4): ``maxiter`` iterations are always enqueued; the stopping test
    ``|f_prev - f| < ftol * f`` clears a device flag that freezes the median, distances and
    weights from the converging iteration on (exactly the values the reference's ``break``
    leaves).  No host sync inside the loop: one read of the per-iteration objectives at the
    end (for the reference's log lines).  ``avg(w)``: weighted sum of the points for the
    normalised fp64 weights ``w`` (device); ``dists(m)``: fp64 distances of the points to m.
    ``poll`` > 0: read the flag every ``poll`` iterations and stop enqueueing once converged
    (the distributed form: each further iteration is two all-reduces; every rank reads the
    same all-reduced objective, so all stop at the same iteration).  Returns (median,
    distances, weights, iterations run = the reference's num_oracle_calls - 1)."""
    dev = alphas.device
    median = avg(alphas)
    d = dists(median)
    obj = (alphas * d).sum()
    active = torch.ones((), dtype=torch.bool, device=dev)
    weights = alphas.clone()
    wv = None
    hist = torch.zeros(maxiter, 3, dtype=torch.float64, device=dev)   # prev_obj, obj, logged
    for i in range(maxiter):
        w = alphas / torch.clamp(d, min=eps)
        w = w / w.sum()
        m_new = avg(w)
        d_new = dists(m_new)
        o_new = (alphas * d_new).sum()
        conv = (obj - o_new).abs() < ftol * o_new
        hist[i, 0], hist[i, 1] = obj, o_new
        hist[i, 2] = (active & ~conv).double()
        weights = torch.where(active, w, weights)
        median = torch.where(active, m_new, median)
        d = torch.where(active, d_new, d)
        obj = torch.where(active, o_new, obj)
        # wv = the weights of the last iteration that did NOT converge (D5: the current ones)
        upd = active & ~conv
        wv = torch.where(upd, w, wv) if wv is not None else torch.where(upd, w, torch.full_like(w, float("nan")))
        active = active & ~conv
        if poll > 0 and (i + 1) % poll == 0 and i + 1 < maxiter and not bool(active.item()):
            break
    h = hist.cpu().numpy()                       # the one host read of the aggregation
    for i in range(maxiter):
        if h[i, 2] > 0:
            log.info(f"[rfa agg] iter:  {i}, prev_obj_val: {h[i, 0]}, obj_val: {h[i, 1]}, "
                     f"abs dis: {abs(h[i, 0] - h[i, 1])}")
    wv_h = wv.cpu().numpy() if wv is not None else None
    if wv_h is None or np.isnan(wv_h).any():      # D5: converged at iteration 0
        wv_h = weights.cpu().numpy()
    # iterations the reference runs: up to and including the converging one (its break)
    iters = min(int((h[:, 2] > 0).sum()) + 1, maxiter)
    return median, d, wv_h, iters


def geometric_median(global_state: torch.Tensor, finals: torch.Tensor, num_samples: Sequence[int],
                     eta: float, maxiter: int, dp: bool, sigma: float, seed: int, n_update: int,
                     eps: float = 1e-5, ftol: float = 1e-6,
                     max_update_norm: Optional[float] = None) -> Tuple[bool, List[float], List[float], int]:
    """Weiszfeld geometric median of the client deltas; returns (updated, wv, alphas, oracle calls)."""
    points = finals[:, :n_update] - global_state[None, :n_update]
    a = torch.tensor(num_samples, dtype=torch.float64, device=points.device)
    alphas = a / a.sum()
    E = fixed_exponent(max_abs(points), points.shape[0])

    def avg(w: torch.Tensor) -> torch.Tensor:
        # exact fixed-point sum of the products (each quantised on its own): the bits the
        # distributed form reaches from its rank partials
        return wsum_decode(wsum_part(points, w / w.sum(), E), E)

    def dists(m: torch.Tensor) -> torch.Tensor:
        return ops.sq_dists(points, m).double().clamp(min=0.0).sqrt()

    median, d, wv, iters = _weiszfeld(avg, dists, alphas, maxiter, eps, ftol)
    return _rfa_apply(global_state, median, d, wv, eta, dp, sigma, seed, n_update, max_update_norm, iters)


def _rfa_apply(global_state, median, d, wv, eta, dp, sigma, seed, n_update, max_update_norm, iters):
    upd_norm = float(torch.linalg.vector_norm(median.double()).item())
    if max_update_norm is None or upd_norm < max_update_norm:
        ops.add_noise_scaled(global_state[:n_update], median, eta, sigma, seed, dp)
        updated = True
    else:
        log.info(f"\t\t\tUpdate norm = {upd_norm} is too large. Update rejected")
        updated = False
    return updated, [float(x) for x in wv], [float(x) for x in d.cpu().tolist()], 1 + iters


def geometric_median_distributed(global_state: torch.Tensor, local_finals: torch.Tensor, local_idx: Sequence[int],
                                 num_samples: Sequence[int], eta: float, maxiter: int, dp: bool, sigma: float,
                                 seed: int, n_update: int, reduce, reduce_max=None, eps: float = 1e-5,
                                 ftol: float = 1e-6, max_update_norm: Optional[float] = None
                                 ) -> Tuple[bool, List[float], List[float], int]:
    """Weiszfeld with the client deltas resident on their owner ranks (reference
    ``helper.py:320-352``): per iteration each rank forms its partial weighted sum of its own
    points as fixed-point limbs (``reduce`` = all-reduce of the [2, S] int64 limbs: exact, so the
    median's bits equal :func:`geometric_median`'s at any world size) and its points' distances
    to the median (all-reduce of an n-vector with zeros for other ranks' clients: exact).
    ``reduce_max``: max-all-reduce of a host float (the fixed grid's exponent: the max |delta|
    over all clients).  Same device-side iteration control and stopping rule."""
    n = len(num_samples)
    dev = global_state.device
    idx = list(local_idx)
    points = local_finals[:, :n_update] - global_state[None, :n_update] if idx else None
    a = torch.tensor(num_samples, dtype=torch.float64, device=dev)
    alphas = a / a.sum()
    idx_t = torch.tensor(idx, dtype=torch.int64, device=dev) if idx else None
    mx = max_abs(points)
    E = fixed_exponent(reduce_max(mx) if reduce_max is not None else mx, n)

    def avg(w: torch.Tensor) -> torch.Tensor:
        wn = w / w.sum()
        part = wsum_part(points, wn[idx_t], E) if idx else wsum_zero(n_update, E, dev)
        return wsum_decode(reduce(part), E)

    def dists(m: torch.Tensor) -> torch.Tensor:
        full = torch.zeros(n, dtype=torch.float64, device=dev)
        if idx:
            full[idx_t] = ops.sq_dists(points, m).double()
        return reduce(full).clamp(min=0.0).sqrt()

    median, d, wv, iters = _weiszfeld(avg, dists, alphas, maxiter, eps, ftol, poll=2)
    return _rfa_apply(global_state, median, d, wv, eta, dp, sigma, seed, n_update, max_update_norm, iters)


class FoolsGold:
    """FoolsGold with per-client history (reference helper.py:527-607)."""

    def __init__(self, use_memory: bool) -> None:
        self.use_memory = use_memory
        self.memory_dict: Dict[str, np.ndarray] = {}
        self.wv_history: List[np.ndarray] = []

    @staticmethod
    def weights(feats: torch.Tensor) -> Tuple[np.ndarray, np.ndarray]:
        """FoolsGold weighting from the [n, d] feature matrix; the cosine Gram F F^T runs on
        the features' device (the MFMA Gram kernel on GPU), the n x n logic on the host."""
        n = feats.shape[0]
        g = ops.gram(feats).double().cpu()
        nrm = torch.sqrt(torch.clamp(torch.diagonal(g), min=0.0))
        nrm = torch.where(nrm == 0, torch.ones_like(nrm), nrm)   # sklearn normalises zero rows to 0
        cs = (g / nrm[:, None] / nrm[None, :]).numpy() - np.eye(n)
        return FoolsGold._from_cs(cs)

    @staticmethod
    def _from_cs(cs: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        n = cs.shape[0]
        cs = cs.copy()
        maxcs = np.max(cs, axis=1)
        for i in range(n):                      # pardoning
            for j in range(n):
                if i == j:
                    continue
                if maxcs[i] < maxcs[j]:
                    cs[i][j] = cs[i][j] * maxcs[i] / maxcs[j]
        wv = 1 - (np.max(cs, axis=1))
        wv[wv > 1] = 1
        wv[wv < 0] = 0
        alpha = np.max(cs, axis=1)
        wv = wv / np.max(wv)
        wv[(wv == 1)] = .99
        with np.errstate(divide="ignore", invalid="ignore"):
            wv = (np.log(wv / (1 - wv)) + 0.5)
        wv[(np.isinf(wv) + wv > 1)] = 1
        wv[(wv < 0)] = 0
        return wv, alpha

    def aggregate(self, grads: torch.Tensor, names: Sequence[Any], feat_slice: Tuple[int, int]
                  ) -> Tuple[torch.Tensor, np.ndarray, np.ndarray]:
        """grads [n, P] summed client gradients -> (aggregated [P], wv, alpha)."""
        lo, hi = feat_slice
        wv, alpha = self.weights_from(grads[:, lo:hi], names)
        wts = torch.tensor(wv / len(names), dtype=torch.float32, device=grads.device)
        E = fixed_exponent(max_abs(grads), len(names))
        agg = wsum_decode(wsum_part(grads, wts, E), E)
        return agg, wv, alpha

    def weights_from(self, feat_rows: torch.Tensor, names: Sequence[Any]) -> Tuple[np.ndarray, np.ndarray]:
        """FoolsGold weights from this round's [n, d] final-layer gradient features (the
        reference's ``client_grads[i][-2]``, ``helper.py:544``): history update, cosine Gram,
        pardoning, logit.  Deterministic, so every rank computes the same weights."""
        feats = feat_rows.double().cpu().numpy()
        mem = np.zeros_like(feats)
        for i, nm in enumerate(names):
            key = str(nm)
            if key in self.memory_dict:
                self.memory_dict[key] = self.memory_dict[key] + feats[i]
            else:
                self.memory_dict[key] = feats[i].copy()
            mem[i] = self.memory_dict[key]
        use = mem if self.use_memory else feats
        wv, alpha = self.weights(torch.from_numpy(use).to(feat_rows.device, torch.float32))
        self.wv_history.append(wv)
        return wv, alpha

    def state(self) -> Dict[str, Any]:
        return {"memory": {k: torch.from_numpy(v) for k, v in self.memory_dict.items()}}

    def load_state(self, st: Dict[str, Any]) -> None:
        self.memory_dict = {k: v.double().numpy() for k, v in st.get("memory", {}).items()}


def foolsgold_server_step(global_state: torch.Tensor, agg: torch.Tensor, P: int, eta: float, lr: float,
                          wd: float) -> None:
    """Fresh ``SGD(lr, momentum, wd)`` single step with ``p.grad = eta * agg``
    (helper.py:280-290): first momentum step means buf = d_p, so p -= lr (eta*agg + wd*p)."""
    p = global_state[:P]
    p -= lr * (eta * agg + wd * p)
