"""Aggregation math vs small numpy oracles written from SURVEY Appendix B (and, for
FoolsGold, vs the reference's sklearn-based formulation)."""
import numpy as np
import pytest
import torch

from dba_mod_amd.fl import aggregate as agg


def test_fedavg_unweighted_with_eta():
    g = torch.randn(100)
    finals = g[None] + torch.randn(4, 100) * 0.1
    g_ref = g.clone() + (0.1 / 10) * (finals - g[None]).sum(0)
    agg.fedavg(g, finals, eta=0.1, no_models=10, dp=False, sigma=0.0, seed=0, n_update=100)
    torch.testing.assert_close(g, g_ref)


def test_fedavg_partial_update_and_dp_noise():
    g = torch.zeros(1000)
    finals = torch.ones(2, 1000)
    agg.fedavg(g, finals, eta=1.0, no_models=2, dp=True, sigma=0.5, seed=7, n_update=600)
    assert torch.all(g[600:] == 0)
    noise = g[:600] - 1.0
    assert abs(noise.mean().item()) < 0.1 and abs(noise.std().item() - 0.5) < 0.06


def _weiszfeld_oracle(points, alphas, maxiter, eps=1e-5, ftol=1e-6):
    alphas = np.asarray(alphas, float) / np.sum(alphas)
    med = (alphas[:, None] * points).sum(0) / alphas.sum()
    obj = sum(a * np.linalg.norm(med - p) for a, p in zip(alphas, points))
    wv = None
    calls = 1
    for _ in range(maxiter):
        prev = obj
        calls += 1
        w = np.array([a / max(eps, np.linalg.norm(med - p)) for a, p in zip(alphas, points)])
        w = w / w.sum()
        med = (w[:, None] * points).sum(0) / w.sum()
        obj = sum(a * np.linalg.norm(med - p) for a, p in zip(alphas, points))
        if abs(prev - obj) < ftol * obj:
            break
        wv = w
    return med, wv, [np.linalg.norm(med - p) for p in points], calls


def test_geometric_median_matches_oracle():
    rng = np.random.RandomState(0)
    pts = rng.randn(6, 50)
    pts[5] += 20.0                      # an outlier the median should resist
    ns = [100, 200, 50, 80, 120, 300]
    g = torch.zeros(50)
    finals = torch.from_numpy(pts).float()
    updated, wv, alphas, calls = agg.geometric_median(g, finals, ns, eta=1.0, maxiter=10, dp=False, sigma=0,
                                                      seed=0, n_update=50)
    med, wv_ref, al_ref, calls_ref = _weiszfeld_oracle(pts, ns, 10)
    # the reference's num_oracle_calls: 1 + the iterations up to its break (helper.py:321-349)
    assert calls == calls_ref
    g2 = torch.zeros(50)
    calls2 = agg.geometric_median(g2, finals, ns, eta=1.0, maxiter=200, dp=False, sigma=0, seed=0, n_update=50)[3]
    assert calls2 == _weiszfeld_oracle(pts, ns, 200)[3] < 201   # converged early: the break's count
    np.testing.assert_allclose(g.numpy(), med, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(wv, wv_ref, rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(alphas, al_ref, rtol=1e-4)
    assert updated and wv[5] < min(wv[:5])


def _foolsgold_sklearn_style(grads):
    # reference helper.py:574-607 semantics (cosine via explicit normalisation)
    n = grads.shape[0]
    nrm = np.linalg.norm(grads, axis=1, keepdims=True)
    nrm[nrm == 0] = 1
    g = grads / nrm
    cs = g @ g.T - np.eye(n)
    maxcs = np.max(cs, axis=1)
    for i in range(n):
        for j in range(n):
            if i != j and maxcs[i] < maxcs[j]:
                cs[i][j] = cs[i][j] * maxcs[i] / maxcs[j]
    wv = 1 - np.max(cs, axis=1)
    wv[wv > 1] = 1
    wv[wv < 0] = 0
    alpha = np.max(cs, axis=1)
    wv = wv / np.max(wv)
    wv[wv == 1] = .99
    with np.errstate(divide="ignore"):
        wv = np.log(wv / (1 - wv)) + 0.5
    wv[(np.isinf(wv) + wv > 1)] = 1
    wv[wv < 0] = 0
    return wv, alpha


def test_foolsgold_weights_and_sybil_suppression():
    rng = np.random.RandomState(1)
    honest = rng.randn(6, 40)
    sybil = rng.randn(1, 40)
    feats = np.concatenate([honest, sybil + 0.01 * rng.randn(3, 40)])   # 3 near-identical sybils
    wv, alpha = agg.FoolsGold.weights(torch.from_numpy(feats).float())
    wv_ref, alpha_ref = _foolsgold_sklearn_style(feats)
    np.testing.assert_allclose(wv, wv_ref, atol=1e-4)
    np.testing.assert_allclose(alpha, alpha_ref, atol=1e-5)
    assert np.all(wv[6:] == 0) and np.all(wv[:6] > 0)


def test_foolsgold_history_and_server_step():
    fg = agg.FoolsGold(use_memory=True)
    P = 30
    grads = torch.randn(3, P)
    a1, wv1, _ = fg.aggregate(grads, ["a", "b", "c"], (10, 20))
    a2, wv2, _ = fg.aggregate(grads, ["a", "b", "d"], (10, 20))
    assert np.allclose(fg.memory_dict["a"], 2 * grads[0, 10:20].double().numpy())
    torch.testing.assert_close(a1, (torch.tensor(wv1 / 3, dtype=torch.float32)[:, None] * grads).sum(0))
    p = torch.randn(P + 5)
    p0 = p.clone()
    agg.foolsgold_server_step(p, a1, P, eta=0.5, lr=0.1, wd=1e-3)
    torch.testing.assert_close(p[:P], p0[:P] - 0.1 * (0.5 * a1 + 1e-3 * p0[:P]))
    assert torch.equal(p[P:], p0[P:])                                   # BN buffers untouched
    st = fg.state()
    fg2 = agg.FoolsGold(True)
    fg2.load_state(st)
    assert set(fg2.memory_dict) == {"a", "b", "c", "d"}


def test_plan_multistep_lr_quirk():
    from dba_mod_amd.fl.plan import _multistep_lrs
    assert _multistep_lrs(1.0, 6, False) == [1.0] * 6            # float milestones 1.2/4.8 never fire
    l10 = _multistep_lrs(1.0, 10, False)
    assert l10[:2] == [1.0, 1.0] and abs(l10[2] - 0.1) < 1e-12 and abs(l10[8] - 0.01) < 1e-12
    l5 = _multistep_lrs(1.0, 5, True)                               # LOAN steps the scheduler first
    assert abs(l5[0] - 0.1) < 1e-12 and abs(l5[-1] - 0.01) < 1e-12


def test_dist_loss_grad_matches_autograd():
    """reference.dist_loss_grad == autograd of a*CE + (1-a)*||w - w_g|| (helper.py:111-123)."""
    from dba_mod_amd.ops import reference as R
    torch.manual_seed(0)
    G, P, S = 3, 300, 320
    w = torch.randn(G, S, dtype=torch.float64)
    base = w + 0.1 * torch.randn(G, S, dtype=torch.float64)
    base[2] = w[2]
    ce_grad = torch.randn(G, P, dtype=torch.float64)
    trig = torch.tensor([1, -1, 0], dtype=torch.int32)
    act = torch.ones(G, dtype=torch.int32)
    alpha = 0.6
    got = ce_grad.clone()
    dist = R.dist_loss_grad(w, base, got, trig, act, alpha)
    for g in range(G):
        wv = w[g, :P].clone().requires_grad_(True)
        lin = (ce_grad[g] * wv).sum()               # d(lin)/dw = ce_grad
        if int(trig[g]) >= 0:
            sv = torch.zeros(P, dtype=torch.float64)
            sv[:] = wv - base[g, :P]
            loss = alpha * lin + (1 - alpha) * torch.norm(sv, 2)
        else:
            loss = lin
        loss.backward()
        assert torch.allclose(got[g], wv.grad, atol=1e-10), g
    assert float(dist[1]) == 0.0 and float(dist[2]) == 0.0
    assert abs(float(dist[0]) - float(torch.norm(w[0, :P] - base[0, :P]))) < 1e-6


def test_fixed_point_weighted_sum_is_order_free():
    """The RFA / FoolsGold weighted sum on the fixed two-limb grid: any split of the clients
    into rank partials (int64 sums, then added) gives the SAME limbs as one pass, in any client
    order — what makes the distributed aggregation world-invariant — and the decoded value is
    the fp64 sum to ~1e-15."""
    from dba_mod_amd.ops import reference as R
    g = torch.Generator().manual_seed(0)
    n, L = 10, 5000
    pts = torch.randn(n, L, generator=g) * torch.exp(3 * torch.randn(n, 1, generator=g))
    pts[3, :100] *= 1e-9                                   # a wide dynamic range inside a row
    w = torch.rand(n, generator=g)
    w = (w / w.sum()).float()
    E = agg.fixed_exponent(float(pts.abs().max()), n)
    full = R.weighted_sum_fixed(pts, w, E)
    for parts in ([[0, 1, 2, 3, 4], [5, 6, 7, 8, 9]], [[9, 2], [0, 5, 7], [1, 3, 4, 6, 8]]):
        tot = sum(R.weighted_sum_fixed(pts[p], w[p], E) for p in parts)
        assert torch.equal(tot, full)
    perm = torch.randperm(n, generator=g)
    assert torch.equal(R.weighted_sum_fixed(pts[perm], w[perm], E), full)
    ref = (w.double()[:, None] * pts.double()).sum(0)
    dec = agg.fixed_decode(full, E)
    assert ((dec - ref).abs().max() / ref.abs().max()).item() < 1e-14
    assert agg.fixed_exponent(0.0, n) == 0


def test_weighted_sum_non_finite_or_many_terms_falls_back_to_fp64():
    """A NaN / Inf client update cannot be put on the fixed grid (it would become finite
    garbage): the exponent is None and the fp64 sum carries the NaN into the aggregate, as the
    reference's torch sum does; more than 512 terms also take the fp64 sum instead of failing."""
    assert agg.fixed_exponent(float("nan"), 10) is None
    assert agg.fixed_exponent(float("inf"), 10) is None
    assert agg.fixed_exponent(1.0, 513) is None and agg.fixed_exponent(1.0, 512) is not None
    pts = torch.randn(4, 300)
    pts[2, 7] = float("nan")
    assert agg.max_abs(pts) == float("inf")
    w = torch.full((4,), 0.25)
    E = agg.fixed_exponent(agg.max_abs(pts), 4)
    out = agg.wsum_decode(agg.wsum_part(pts, w, E), E)
    assert torch.isnan(out[7]) and torch.isfinite(out[:7]).all()
    # RFA end to end: the NaN reaches the global model
    g = torch.zeros(300)
    finals = g[None] + pts
    agg.geometric_median(g, finals, [10, 10, 10, 10], 1.0, 3, False, 0.0, 1, 300)
    assert torch.isnan(g).any()
    # FoolsGold's weighted sum over 600 clients: the fp64 path, equal to the plain sum
    many = torch.randn(600, 50, dtype=torch.float64).float()
    wm = torch.rand(600)
    E = agg.fixed_exponent(agg.max_abs(many), 600)
    got = agg.wsum_decode(agg.wsum_part(many, wm, E), E)
    ref = (wm.double()[:, None] * many.double()).sum(0).float()
    assert torch.equal(got, ref)
