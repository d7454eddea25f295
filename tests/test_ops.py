"""Numerics of the stand-alone device ops (lightgbmv1_amd.ops -> src/capi/ops_api.cpp ->
the HIP kernels of src/device/) against plain PyTorch float64 references of the same op:
objective gradients (reference src/objective/*.hpp GetGradients), metrics (reference
src/metric/*.hpp) and the bagging sampler (reference gbdt.cpp:162-243, Random = LCG
214013 / 2531011)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

N = 5000


def _data(seed=0, kind="reg"):
    rng = np.random.RandomState(seed)
    score = rng.randn(N)
    if kind == "bin":
        y = (rng.rand(N) > 0.6).astype(np.float32)
    elif kind == "pos":
        y = rng.gamma(2.0, 1.5, N).astype(np.float32) + 0.1
    elif kind == "prob":
        y = rng.rand(N).astype(np.float32)
    else:
        y = rng.randn(N).astype(np.float32)
    w = (rng.rand(N) + 0.5).astype(np.float32)
    return score, y, w


def _t(a):
    return torch.tensor(a, dtype=torch.float64)


def _ref_grad(obj, s, y, w, params):
    """float64 torch reference of the objective's (grad, hess)."""
    s, y = _t(s), _t(y)
    w = _t(w) if w is not None else torch.ones_like(s)
    if obj == "regression":
        return (s - y) * w, w.clone()
    if obj == "regression_l1":
        return torch.sign(s - y) * w, w.clone()
    if obj == "huber":
        a = params["alpha"]
        d = s - y
        return torch.where(d.abs() <= a, d, torch.sign(d) * a) * w, w.clone()
    if obj == "fair":
        c = params["fair_c"]
        x = s - y
        return c * x / (x.abs() + c) * w, c * c / (x.abs() + c) ** 2 * w
    if obj == "poisson":
        return (torch.exp(s) - y) * w, torch.exp(s + params["poisson_max_delta_step"]) * w
    if obj == "quantile":
        a = params["alpha"]
        return torch.where(s - y >= 0, 1 - a, -a) * w, w.clone()
    if obj == "gamma":
        return 1.0 - y / torch.exp(s) * w, y / torch.exp(s) * w
    if obj == "tweedie":
        r = params["tweedie_variance_power"]
        e1, e2 = torch.exp((1 - r) * s), torch.exp((2 - r) * s)
        return (-y * e1 + e2) * w, (-y * (1 - r) * e1 + (2 - r) * e2) * w
    if obj == "binary":
        sig = params.get("sigmoid", 1.0)
        lab = torch.where(y > 0, 1.0, -1.0).double()
        resp = -lab * sig / (1 + torch.exp(lab * sig * s))
        return resp * w, resp.abs() * (sig - resp.abs()) * w
    if obj == "cross_entropy":
        z = torch.sigmoid(s)
        return (z - y) * w, z * (1 - z) * w
    raise KeyError(obj)


GRAD_CASES = [
    ("regression", "reg", {}), ("regression_l1", "reg", {}), ("huber", "reg", {"alpha": 0.7}),
    ("fair", "reg", {"fair_c": 1.3}), ("poisson", "pos", {"poisson_max_delta_step": 0.7}),
    ("quantile", "reg", {"alpha": 0.3}), ("gamma", "pos", {}), ("tweedie", "pos", {"tweedie_variance_power": 1.4}),
    ("binary", "bin", {"sigmoid": 1.7}), ("cross_entropy", "prob", {}),
]


@pytest.mark.parametrize("obj,kind,params", GRAD_CASES, ids=[c[0] for c in GRAD_CASES])
@pytest.mark.parametrize("weighted", [False, True])
def test_gradients_match_torch(obj, kind, params, weighted, gpu_available):
    from lightgbmv1_amd import ops
    s, y, w = _data(kind=kind)
    w = w if weighted else None
    p = dict(params, objective=obj, verbose=-1)
    g, h = ops.gradients(p, torch.tensor(s, device="cuda"), y, w)
    rg, rh = _ref_grad(obj, s, y, w, params)
    # the kernels compute in float64 and store float32 (score_t)
    np.testing.assert_allclose(g.cpu().double().numpy(), rg.float().double().numpy(), rtol=2e-6, atol=1e-6)
    np.testing.assert_allclose(h.cpu().double().numpy(), rh.float().double().numpy(), rtol=2e-6, atol=1e-6)


def test_gradients_and_bagging_with_poisoned_args(monkeypatch, gpu_available):
    """LGBM_AMD_POISON_ARGS=1 fills the argument structs with 0xA5 bytes before their call sites
    set them: a field the call site forgets reads garbage on every run (round 5's unset
    GradArgs::write_split zeroed the gradients on one box only)."""
    from lightgbmv1_amd import ops
    monkeypatch.setenv("LGBM_AMD_POISON_ARGS", "1")
    for obj, kind, params in GRAD_CASES:
        for weighted in (False, True):
            s, y, w = _data(kind=kind)
            w = w if weighted else None
            g, h = ops.gradients(dict(params, objective=obj, verbose=-1), torch.tensor(s, device="cuda"), y, w)
            rg, rh = _ref_grad(obj, s, y, w, params)
            np.testing.assert_allclose(g.cpu().double().numpy(), rg.float().double().numpy(), rtol=2e-6, atol=1e-6,
                                       err_msg=obj)
            np.testing.assert_allclose(h.cpu().double().numpy(), rh.float().double().numpy(), rtol=2e-6, atol=1e-6,
                                       err_msg=obj)
    bag, oob = ops.sample_rows(10 * 1024 + 77, fraction=0.5, seed=3)
    rb, ro = _ref_bag(10 * 1024 + 77, 0.5, 3)
    np.testing.assert_array_equal(bag.cpu().numpy(), rb)
    np.testing.assert_array_equal(oob.cpu().numpy(), ro)


def test_multiclass_softmax_gradients_match_torch(gpu_available):
    from lightgbmv1_amd import ops
    K = 4
    rng = np.random.RandomState(1)
    score = rng.randn(K, N)
    y = rng.randint(0, K, N).astype(np.float32)
    g, h = ops.gradients({"objective": "multiclass", "num_class": K, "verbose": -1},
                         torch.tensor(score, device="cuda"), y)
    p = torch.softmax(_t(score), dim=0)
    onehot = torch.nn.functional.one_hot(torch.tensor(y, dtype=torch.long), K).T.double()
    rg = p - onehot
    rh = K / (K - 1.0) * p * (1 - p)
    np.testing.assert_allclose(g.cpu().double().numpy(), rg.numpy(), rtol=2e-6, atol=1e-6)
    np.testing.assert_allclose(h.cpu().double().numpy(), rh.numpy(), rtol=2e-6, atol=1e-6)


def _ref_auc(s, y, w):
    """weighted AUC with ties counted one half (Mann-Whitney), float64 torch."""
    s, y, w = _t(s), _t(y), _t(w)
    order = torch.argsort(s)
    s, y, w = s[order], y[order], w[order]
    pos_w = torch.where(y > 0, w, 0.0)
    neg_w = torch.where(y > 0, 0.0, w)
    uniq, inv = torch.unique_consecutive(s, return_inverse=True)
    pw = torch.zeros(len(uniq), dtype=torch.float64).index_add_(0, inv, pos_w)
    nw = torch.zeros(len(uniq), dtype=torch.float64).index_add_(0, inv, neg_w)
    neg_below = torch.cumsum(nw, 0) - nw
    acc = (pw * (neg_below + 0.5 * nw)).sum()
    return float(acc / (pw.sum() * nw.sum()))


@pytest.mark.parametrize("weighted", [False, True])
def test_metrics_match_torch(weighted, gpu_available):
    from lightgbmv1_amd import ops
    s, y, w = _data(kind="bin")
    s = np.round(s, 1)  # plenty of ties for the AUC
    w = w if weighted else None
    ww = w if w is not None else np.ones(N, np.float32)
    ds = torch.tensor(s, device="cuda")
    prob = torch.sigmoid(_t(s))
    tw, ty = _t(ww), _t(y)
    ref = {
        "auc": _ref_auc(s, y, ww),
        "binary_logloss": float((-(ty * torch.log(prob.clamp_min(1e-15)) +
                                   (1 - ty) * torch.log((1 - prob).clamp_min(1e-15))) * tw).sum() / tw.sum()),
        "binary_error": float((((prob > 0.5).double() != ty).double() * tw).sum() / tw.sum()),
    }
    for name, r in ref.items():
        v = ops.metric({"metric": name, "objective": "binary", "verbose": -1}, ds, y, w)
        assert abs(v - r) < 1e-9 * max(1.0, abs(r)), (name, v, r)
    sr, yr, _ = _data(kind="reg")
    dr = torch.tensor(sr, device="cuda")
    d = _t(sr) - _t(yr)
    for name, r in {"l2": float((d * d * tw).sum() / tw.sum()), "l1": float((d.abs() * tw).sum() / tw.sum()),
                    "rmse": float(torch.sqrt((d * d * tw).sum() / tw.sum()))}.items():
        v = ops.metric({"metric": name, "objective": "regression", "verbose": -1}, dr, yr, w)
        assert abs(v - r) < 1e-9 * max(1.0, abs(r)), (name, v, r)


def _ref_bag(n, fraction, seed):
    """the reference's bagging: generator Random(seed + b) per 1024-row block b."""
    keep = np.zeros(n, dtype=bool)
    for b in range((n + 1023) // 1024):
        x = (seed + b) & 0xFFFFFFFF
        for r in range(b * 1024, min(n, (b + 1) * 1024)):
            x = (214013 * x + 2531011) & 0xFFFFFFFF
            keep[r] = ((x >> 16) & 0x7FFF) / 32768.0 < fraction
    return np.nonzero(keep)[0], np.nonzero(~keep)[0]


@pytest.mark.parametrize("fraction,seed", [(0.5, 3), (0.9, 17), (0.1, 12345)])
def test_bagging_matches_reference_generator(fraction, seed, gpu_available):
    from lightgbmv1_amd import ops
    n = 10 * 1024 + 77
    bag, oob = ops.sample_rows(n, fraction=fraction, seed=seed)
    rb, ro = _ref_bag(n, fraction, seed)
    np.testing.assert_array_equal(bag.cpu().numpy(), rb)
    np.testing.assert_array_equal(oob.cpu().numpy(), ro)


def test_goss_keeps_top_rows_and_rescales(gpu_available):
    """GOSS per 1024-row block: the top_rate largest |g*h| are kept as they are, other_rate
    of the rest are sampled and multiplied by (cnt - top_k) / other_k."""
    from lightgbmv1_amd import ops
    n = 4 * 1024
    rng = np.random.RandomState(5)
    g0 = rng.randn(n).astype(np.float32)
    h0 = (rng.rand(n) + 0.1).astype(np.float32)
    g, h = torch.tensor(g0, device="cuda"), torch.tensor(h0, device="cuda")
    bag, _ = ops.sample_rows(n, goss=True, top_rate=0.2, other_rate=0.1, grad=g, hess=h, seed=9)
    bag = bag.cpu().numpy()
    gn, hn = g.cpu().numpy(), h.cpu().numpy()
    top_k, other_k = int(1024 * 0.2), int(1024 * 0.1)
    mult = np.float32(1024 - top_k) / other_k
    for b in range(4):
        rows = np.arange(b * 1024, (b + 1) * 1024)
        wt = np.abs(g0[rows] * h0[rows])
        thr = np.sort(wt)[::-1][top_k - 1]
        top = rows[wt >= thr]
        inbag = bag[(bag >= rows[0]) & (bag <= rows[-1])]
        assert set(top) <= set(inbag)
        small = np.setdiff1d(inbag, top)
        assert len(small) == other_k
        np.testing.assert_allclose(gn[small], g0[small] * mult, rtol=1e-6)
        np.testing.assert_allclose(hn[small], h0[small] * mult, rtol=1e-6)
        np.testing.assert_array_equal(gn[top], g0[top])


def test_regression_family_metrics_match_torch(gpu_available):
    """Point-wise regression / cross-entropy metrics on device scores (with their objective's
    output transform) against float64 torch references of the reference formulas
    (regression_metric.hpp, xentropy_metric.hpp)."""
    from lightgbmv1_amd import ops
    s, y, w = _data(seed=3, kind="reg")
    sp, yp, _ = _data(seed=4, kind="pos")
    sq, yq, _ = _data(seed=5, kind="prob")
    tw = _t(w)

    def wmean(v):
        return float((v * tw).sum() / tw.sum())

    ts, ty = _t(s), _t(y)
    cases = []
    d = ty - ts
    cases.append(({"metric": "quantile", "objective": "quantile", "alpha": 0.7}, s, y,
                  wmean(torch.where(d < 0, (0.7 - 1) * d, 0.7 * d))))
    d = ts - ty
    cases.append(({"metric": "huber", "objective": "huber", "alpha": 0.9}, s, y,
                  wmean(torch.where(d.abs() <= 0.9, 0.5 * d * d, 0.9 * (d.abs() - 0.45)))))
    x = (ts - ty).abs()
    cases.append(({"metric": "fair", "objective": "fair", "fair_c": 1.3}, s, y,
                  wmean(1.3 * x - 1.3 * 1.3 * torch.log1p(x / 1.3))))
    cases.append(({"metric": "mape", "objective": "mape"}, s, y,
                  wmean((ty - ts).abs() / torch.clamp(ty.abs(), min=1.0))))
    p, typ = torch.exp(_t(sp)), _t(yp)
    cases.append(({"metric": "poisson", "objective": "poisson"}, sp, yp, wmean(p - typ * torch.log(p))))
    cases.append(({"metric": "gamma", "objective": "gamma"}, sp, yp, wmean(typ / p + torch.log(p))))
    t = typ / (p + 1e-9)
    cases.append(({"metric": "gamma_deviance", "objective": "gamma"}, sp, yp,
                  2 * float(((t - torch.log(t) - 1) * tw).sum())))
    r = 1.5
    cases.append(({"metric": "tweedie", "objective": "tweedie", "tweedie_variance_power": r}, sp, yp,
                  wmean(-typ * p ** (1 - r) / (1 - r) + p ** (2 - r) / (2 - r))))
    pq, tyq = torch.sigmoid(_t(sq)), _t(yq)
    xent = -(tyq * torch.log(pq.clamp_min(1e-12)) + (1 - tyq) * torch.log((1 - pq).clamp_min(1e-12)))
    cases.append(({"metric": "cross_entropy", "objective": "cross_entropy"}, sq, yq, wmean(xent)))
    ent = tyq * torch.log(tyq) + (1 - tyq) * torch.log(1 - tyq)
    cases.append(({"metric": "kullback_leibler", "objective": "cross_entropy"}, sq, yq, wmean(xent + ent)))
    for params, sc, lab, ref in cases:
        v = ops.metric(dict(params, verbose=-1), torch.tensor(sc, device="cuda"), lab, w)
        assert abs(v - ref) < 1e-8 * max(1.0, abs(ref)), (params["metric"], v, ref)


@pytest.mark.parametrize("objective", ["multiclass", "multiclassova"])
def test_multiclass_metrics_match_torch(objective, gpu_available):
    from lightgbmv1_amd import ops
    K = 4
    rng = np.random.RandomState(7)
    s = rng.randn(K, N)
    y = rng.randint(0, K, N).astype(np.float32)
    w = (rng.rand(N) + 0.5).astype(np.float32)
    ts, tw = _t(s), _t(w)
    prob = torch.softmax(ts, dim=0) if objective == "multiclass" else torch.sigmoid(ts)
    py = prob[_t(y).long(), torch.arange(N)]
    refs = {"multi_logloss": float((-torch.log(py.clamp_min(1e-15)) * tw).sum() / tw.sum())}
    for k in (1, 2):
        larger = (prob >= py.unsqueeze(0)).sum(dim=0)
        refs["multi_error@%d" % k] = float(((larger > k).double() * tw).sum() / tw.sum())
    ds = torch.tensor(s, device="cuda").contiguous()
    for name, ref in refs.items():
        params = {"metric": name.split("@")[0], "objective": objective, "num_class": K, "verbose": -1}
        if "@" in name:
            params["multi_error_top_k"] = int(name.split("@")[1])
        v = ops.metric(params, ds, y, w)
        assert abs(v - ref) < 1e-9 * max(1.0, abs(ref)), (name, v, ref)
