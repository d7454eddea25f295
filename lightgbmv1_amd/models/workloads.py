"""The reference's benchmark workloads as (parameters, synthetic data) pairs.

Each workload is one of the datasets the reference publishes training speed and accuracy
for (reference docs/GPU-Performance.rst:14-60 and :108-125 -- the GPU comparison with its
training configuration -- and docs/Experiments.rst:100-199), with:

* ``params(max_bin)`` -- that configuration (``max_bin`` in {255, 63, 15} as in the
  reference's bin sweep);
* ``make(rows, seed)`` -- synthetic data of the dataset's shape and character (dense /
  sparse / NaN-heavy / categorical / grouped queries), deterministic in ``seed``.  There is
  no network access, so the real datasets are never downloaded; the generators keep the
  properties that decide training speed (rows, features, sparsity, bin structure, query
  sizes) and give a learnable label so quality can be tracked;
* ``reference`` -- the published numbers (GTX 1080 / CPU wall
  time for 500 iterations, test AUC / NDCG).

``bench.py`` (the headline metric) uses the ``higgs`` workload with its own 63-leaf
configuration from BASELINE.json; ``tools/bench_workload.py`` runs any of them.
"""
from dataclasses import dataclass, field
from typing import Callable, Dict, Optional

import numpy as np

# reference docs/GPU-Performance.rst:108-125 (training configuration of the GPU comparison)
_GPU_PERF_PARAMS = {
    "num_leaves": 255,
    "learning_rate": 0.1,
    "min_data_in_leaf": 1,
    "min_sum_hessian_in_leaf": 100,
    "tree_learner": "serial",
    "verbose": -1,
}


@dataclass
class Workload:
    name: str
    task: str                    # "binary" or "ranking"
    rows: int                    # the real dataset's training rows
    features: int
    make: Callable               # (rows, seed) -> (X, y, group or None)
    extra_params: Dict = field(default_factory=dict)
    reference: Dict = field(default_factory=dict)
    categorical: Optional[list] = None

    def params(self, max_bin=63, device="gpu"):
        p = dict(_GPU_PERF_PARAMS, max_bin=max_bin, device_type=device)
        if self.task == "binary":
            p.update(objective="binary", metric="auc")
        else:
            p.update(objective="lambdarank", metric="ndcg", ndcg_eval_at=[1, 3, 5, 10])
        p.update(self.extra_params)
        return p


def make_higgs(rows, seed=20240601, start=0, num_features=28):
    """Higgs-like rows [start, start + rows): 21 "low-level" kinematic features and 7
    "high-level" invariant-mass-like features, non-linear label.  Generated in 2^20-row
    blocks seeded by block index, so any row range (a rank's shard) is reproducible."""
    block = 1 << 20
    X = np.empty((rows, num_features), dtype=np.float32)
    y = np.empty(rows, dtype=np.float32)
    done = 0
    while done < rows:
        gidx = start + done
        b = gidx // block
        off = gidx % block
        n = min(rows - done, block - off)
        rng = np.random.default_rng(seed + b)
        low = rng.standard_normal((block, 21), dtype=np.float32)[off:off + n]
        low[:, 0::3] = np.abs(low[:, 0::3]) * 0.7 + 0.3          # momenta-like (positive, skewed)
        low[:, 1::3] = np.clip(low[:, 1::3], -2.5, 2.5)          # pseudo-rapidities
        low[:, 2::3] = np.tanh(low[:, 2::3]) * 1.74              # angles
        m = np.empty((n, num_features - 21), dtype=np.float32)   # high-level invariant masses
        for j in range(num_features - 21):
            a, c = low[:, (3 * j) % 21], low[:, (3 * j + 3) % 21]
            m[:, j] = np.sqrt(np.abs(a * c * (1.0 + np.cos(low[:, (3 * j + 2) % 21] - low[:, (3 * j + 5) % 21]))))
        X[done:done + n, :21] = low
        X[done:done + n, 21:] = m
        noise = np.random.default_rng(seed + 7919 + b).standard_normal(block, dtype=np.float32)[off:off + n]
        logit = (1.2 * m[:, 0] - 0.8 * m[:, 1] + 0.6 * m[:, 2] * low[:, 0] - 0.5 * low[:, 3] ** 2
                 + 0.4 * np.sin(2.0 * low[:, 4]) + 0.3 * m[:, 3] * m[:, 4] - 0.9 + 0.8 * noise)
        y[done:done + n] = (logit > 0).astype(np.float32)
        done += n
    return X, y, None


def make_epsilon(rows, seed=11, num_features=2000):
    """Epsilon-like: dense, all features informative-ish (unit-norm rows), linear label."""
    rng = np.random.default_rng(seed)
    w = np.random.default_rng(4242).normal(0, 1, num_features).astype(np.float32)
    X = np.empty((rows, num_features), dtype=np.float32)
    y = np.empty(rows, dtype=np.float32)
    chunk = 1 << 15
    for s in range(0, rows, chunk):
        e = min(rows, s + chunk)
        x = rng.standard_normal((e - s, num_features), dtype=np.float32)
        x /= np.linalg.norm(x, axis=1, keepdims=True)
        X[s:e] = x
        logit = 3.0 * (x @ w)  # x has unit norm, so x @ w ~ N(0, 1)
        y[s:e] = (logit + 0.3 * rng.standard_normal(e - s, dtype=np.float32) > 0).astype(np.float32)
    return X, y, None


def make_bosch(rows, seed=13, num_features=968):
    """Bosch-like: production-line measurements, ~80% missing (NaN) per row in station
    blocks, rare positive label (a few percent)."""
    rng = np.random.default_rng(seed)
    stations = 50
    per = num_features // stations
    X = np.full((rows, num_features), np.nan, dtype=np.float32)
    y = np.empty(rows, dtype=np.float32)
    chunk = 1 << 16
    wv = np.random.default_rng(77).normal(0, 1, 30).astype(np.float32)
    for s in range(0, rows, chunk):
        e = min(rows, s + chunk)
        n = e - s
        visit = rng.random((n, stations)) < 0.2
        vals = np.round(rng.standard_normal((n, num_features), dtype=np.float32), 3)
        mask = np.repeat(visit, per, axis=1)
        mask = np.concatenate([mask, np.zeros((n, num_features - mask.shape[1]), bool)], axis=1)
        blk = X[s:e]
        blk[mask] = vals[mask]
        score = np.nan_to_num(blk[:, :30]) @ wv + 1.5 * visit[:, 3] - 5.2
        y[s:e] = (rng.random(n) < 1 / (1 + np.exp(-score))).astype(np.float32)
    return X, y, None


def _queries(rows, rng, lo, hi, div):
    # rows // div draws: div well below the mean query size covers the rows
    sizes = rng.integers(lo, hi + 1, size=rows // div + 16)
    cum = np.cumsum(sizes)
    nq = int(np.searchsorted(cum, rows)) + 1
    sizes = sizes[:nq].copy()
    sizes[-1] -= int(cum[nq - 1] - rows)
    return sizes


def make_ltr(rows, seed=7, num_features=137, informative=40, query_size=(20, 220), sparse_share=0.4,
             query_div=60):
    """MS-LTR-like learning to rank: queries of 20-220 documents, ``informative`` dense
    relevance features, the rest dense noise and sparse count features; graded relevance
    0-4 (a relevance function shared across seeds, so held-out sets are comparable)."""
    rng = np.random.default_rng(seed)
    sizes = _queries(rows, rng, query_size[0], query_size[1], query_div)
    qid = np.repeat(np.arange(len(sizes)), sizes)
    q_off = rng.normal(0.0, 0.7, size=len(sizes)).astype(np.float32)
    w = np.random.default_rng(12345).normal(0.0, 1.0, size=informative).astype(np.float32) / np.sqrt(informative)
    X = np.empty((rows, num_features), dtype=np.float32)
    rel = np.empty(rows, dtype=np.float32)
    chunk = 1 << 19
    n_dense = informative + int((num_features - informative) * (1.0 - sparse_share))
    for s in range(0, rows, chunk):
        e = min(rows, s + chunk)
        n = e - s
        inf = rng.standard_normal((n, informative), dtype=np.float32)
        X[s:e, :informative] = inf
        X[s:e, informative:n_dense] = rng.standard_normal((n, n_dense - informative), dtype=np.float32)
        X[s:e, n_dense:] = rng.poisson(0.15, size=(n, num_features - n_dense)).astype(np.float32)
        rel[s:e] = inf @ w + q_off[qid[s:e]] + 0.6 * rng.standard_normal(n, dtype=np.float32)
    cuts = np.quantile(rel, [0.50, 0.80, 0.95, 0.98])
    y = np.searchsorted(cuts, rel).astype(np.float32)
    return X, y, sizes


def make_yahoo(rows, seed=9):
    """Yahoo-LTR-like: 700 features, most of them sparse (zero for most documents), queries
    of ~5-50 documents."""
    return make_ltr(rows, seed, num_features=700, informative=60, query_size=(5, 45), sparse_share=0.85,
                    query_div=5)


def make_expo(rows, seed=17, num_features=700, num_cat=8):
    """Expo-like (airline delays): a few high-cardinality categorical columns (integer
    codes) plus one-hot-like sparse indicators; ~20% positive label."""
    rng = np.random.default_rng(seed)
    X = np.zeros((rows, num_features), dtype=np.float32)
    y = np.empty(rows, dtype=np.float32)
    card = [12, 31, 7, 24, 300, 300, 20, 50][:num_cat]
    eff = [np.random.default_rng(500 + j).normal(0, 0.6, c).astype(np.float32) for j, c in enumerate(card)]
    chunk = 1 << 18
    for s in range(0, rows, chunk):
        e = min(rows, s + chunk)
        n = e - s
        logit = np.full(n, -1.6, dtype=np.float32)
        for j, c in enumerate(card):
            code = rng.integers(0, c, n)
            X[s:e, j] = code
            logit += eff[j][code]
        hot = rng.integers(num_cat, num_features, size=(n, 6))
        rows_idx = np.repeat(np.arange(n), 6)
        X[s:e][rows_idx, hot.reshape(-1)] = 1.0
        y[s:e] = (rng.random(n) < 1 / (1 + np.exp(-logit))).astype(np.float32)
    return X, y, None


def make_criteo(rows, seed=5):
    """Criteo-like CTR: 13 heavy-tailed count features and 54 sparse count-encoded
    categorical features (reference docs/Experiments.rst:190-199, 67 features)."""
    rng = np.random.default_rng(seed)
    X = np.zeros((rows, 67), dtype=np.float32)
    y = np.empty(rows, dtype=np.float32)
    wd = np.random.default_rng(99).normal(0, 0.35, size=13).astype(np.float32)
    ws = np.random.default_rng(98).normal(0, 0.8, size=54).astype(np.float32)
    dens = np.random.default_rng(97).uniform(0.005, 0.03, size=54)
    chunk = 1 << 21
    for s in range(0, rows, chunk):
        e = min(rows, s + chunk)
        n = e - s
        d = np.floor(rng.pareto(1.5, size=(n, 13)).astype(np.float32) * 3.0)
        X[s:e, :13] = d
        logit = np.log1p(d) @ wd - 3.6
        for j in range(54):
            nz = rng.random(n) < dens[j]
            cnt = nz.sum()
            if cnt:
                v = np.floor(rng.pareto(1.2, size=cnt).astype(np.float32) * 5.0) + 1.0
                X[s:e, 13 + j][nz] = v
                logit[nz] += ws[j] * np.log1p(v)
        y[s:e] = (rng.random(n) < 1.0 / (1.0 + np.exp(-logit))).astype(np.float32)
    return X, y, None


# published numbers: GTX 1080 wall time for 500 iterations at 255 / 63 / 15 bins and the
# CPU (28-core) time at 255 bins, test quality
WORKLOADS = {
    "higgs": Workload("higgs", "binary", 10_500_000, 28, make_higgs,
                      reference={"gtx1080_s_500it": {255: 116, 63: 112, 15: 104}, "cpu_s_500it_255": 291,
                                 "auc": 0.845612}),
    "epsilon": Workload("epsilon", "binary", 400_000, 2000, make_epsilon,
                        reference={"gtx1080_s_500it": {255: 360, 63: 165, 15: 83}, "cpu_s_500it_255": 1389,
                                   "auc": 0.950243}),
    "bosch": Workload("bosch", "binary", 1_000_000, 968, make_bosch,
                      extra_params={"learning_rate": 0.015, "min_sum_hessian_in_leaf": 5},
                      reference={"gtx1080_s_500it": {255: 161, 63: 108, 15: 68}, "cpu_s_500it_255": 761,
                                 "auc": 0.718115}),
    "ms_ltr": Workload("ms_ltr", "ranking", 2_270_296, 137, make_ltr,
                       reference={"gtx1080_s_500it": {255: 123, 63: 111, 15: 102}, "cpu_s_500it_255": 215,
                                  "ndcg@10": 0.527835}),
    "expo": Workload("expo", "binary", 11_000_000, 700, make_expo, categorical=list(range(8)),
                     reference={"gtx1080_s_500it": {255: 86, 63: 85, 15: 85}, "cpu_s_500it_255": 176,
                                "auc": 0.776217}),
    "yahoo_ltr": Workload("yahoo_ltr", "ranking", 473_134, 700, make_yahoo,
                          reference={"gtx1080_s_500it": {255: 101, 63: 65, 15: 49}, "cpu_s_500it_255": 146,
                                     "ndcg@10": 0.79655}),
    "criteo": Workload("criteo", "binary", 1_700_000_000, 67, make_criteo,
                       extra_params={"min_data_in_leaf": 20},
                       reference={"cpu_s_per_tree_1_machine": 627.8, "cpu_s_per_tree_8_machines": 80.0}),
}


def get(name):
    if name not in WORKLOADS:
        raise KeyError("unknown workload %r (known: %s)" % (name, ", ".join(sorted(WORKLOADS))))
    return WORKLOADS[name]
