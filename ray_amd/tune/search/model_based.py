"""Model-based searchers implemented natively on numpy.

The reference ships these as thin adapters over third-party libraries
(python/ray/tune/search/hyperopt/hyperopt_search.py:HyperOptSearch,
python/ray/tune/search/optuna/optuna_search.py:OptunaSearch,
python/ray/tune/search/bayesopt/bayesopt_search.py:BayesOptSearch).  None of those
libraries are in this image, so the underlying algorithms are implemented here directly:

* ``TPESearch`` -- Tree-structured Parzen Estimator (Bergstra et al. 2011), the default
  algorithm of both HyperOpt and Optuna.  ``HyperOptSearch`` and ``OptunaSearch`` are
  provided as names for it so reference code keeps working; they accept the same
  ``space``/``metric``/``mode``/``points_to_evaluate`` arguments but none of the
  library-specific space formats.
* ``BayesOptSearch`` -- Gaussian-process regression (Matern-5/2 kernel) with UCB / EI /
  PI acquisition over a continuous box, like the ``bayes_opt`` package behind the
  reference adapter.

Every searcher works on the Tune search-space primitives in ``sample.py`` (nested dicts are
supported; constants pass through) and follows the ``Searcher`` contract of
python/ray/tune/search/searcher.py: ``suggest(trial_id) -> config | None`` and
``on_trial_complete(trial_id, result)``.
"""

from __future__ import annotations

import copy
import math

import numpy as np

from ray_amd.tune.search.sample import Categorical, Float, Function, Grid, Integer, _set, _walk
from ray_amd.tune.tuner import Searcher


class _Space:
    """Maps Tune domains onto the unit cube (numeric) and index sets (categorical)."""

    def __init__(self, space: dict):
        self.space = space
        self.params = []
        for path, dom in _walk(space):
            if isinstance(dom, (Grid, Function)):
                raise ValueError(f"model-based searchers do not support {type(dom).__name__} "
                                 f"at {'/'.join(map(str, path))}; use BasicVariantGenerator")
            if isinstance(dom, Float) and dom.normal is not None:
                mu, sd = dom.normal
                dom = Float(mu - 4 * sd, mu + 4 * sd, q=dom.q)
            self.params.append((path, dom))
        if not self.params:
            raise ValueError("search space has no sampled parameters")

    def is_numeric(self, i):
        return not isinstance(self.params[i][1], Categorical)

    def n_choices(self, i):
        return len(self.params[i][1].categories)

    def to_unit(self, i, v):
        dom = self.params[i][1]
        if isinstance(dom, Categorical):
            return float(dom.categories.index(v))
        lo, hi = dom.lower, dom.upper
        if dom.log:
            return (math.log(v) - math.log(lo)) / max(math.log(hi) - math.log(lo), 1e-12)
        return (v - lo) / max(hi - lo, 1e-12)

    def from_unit(self, i, u):
        dom = self.params[i][1]
        if isinstance(dom, Categorical):
            return dom.categories[int(u)]
        u = min(max(float(u), 0.0), 1.0)
        lo, hi = dom.lower, dom.upper
        v = math.exp(math.log(lo) + u * (math.log(hi) - math.log(lo))) if dom.log else \
            lo + u * (hi - lo)
        if dom.q:
            v = round(v / dom.q) * dom.q
        if isinstance(dom, Integer):
            # reference Integer upper bound is exclusive (randint semantics)
            v = int(min(max(round(v), lo), max(hi - 1, lo)))
        return v

    def encode(self, cfg: dict):
        out = []
        for i, (path, _) in enumerate(self.params):
            v = cfg
            for p in path:
                v = v[p]
            out.append(self.to_unit(i, v))
        return np.asarray(out, dtype=np.float64)

    def decode(self, x) -> dict:
        cfg = copy.deepcopy(self.space)
        for i, (path, _) in enumerate(self.params):
            _set(cfg, path, self.from_unit(i, x[i]))
        return cfg


class _ModelSearcher(Searcher):
    def __init__(self, space=None, metric=None, mode=None, points_to_evaluate=None, seed=None):
        super().__init__(metric, mode)
        self._space = _Space(space) if space else None
        self._points = list(points_to_evaluate or [])
        self._rng = np.random.default_rng(seed)
        self._live: dict[str, np.ndarray] = {}
        self.X: list[np.ndarray] = []
        self.y: list[float] = []   # always "lower is better" internally

    def set_search_properties(self, metric, mode, config):
        super().set_search_properties(metric, mode, config)
        if self._space is None and config:
            self._space = _Space(config)
        return True

    def suggest(self, trial_id):
        if self._space is None:
            raise RuntimeError(f"{type(self).__name__} needs a search space (pass space= or "
                               "Tuner(param_space=...))")
        if self._points:
            p = self._points.pop(0)
            cfg = self._space.decode(self._space.encode(_merge(self._space.space, p)))
        else:
            cfg = self._space.decode(self._propose())
        self._live[trial_id] = self._space.encode(cfg)
        return cfg

    def on_trial_complete(self, trial_id, result=None, error=False):
        x = self._live.pop(trial_id, None)
        if x is None or error or not result or self.metric not in result:
            return
        v = float(result[self.metric])
        if not math.isfinite(v):
            return
        self.X.append(x)
        self.y.append(-v if self.mode == "max" else v)

    def _random(self):
        sp = self._space
        return np.array([self._rng.uniform() if sp.is_numeric(i) else
                         float(self._rng.integers(sp.n_choices(i)))
                         for i in range(len(sp.params))])

    def _propose(self):
        raise NotImplementedError

    # reference Searcher.save/restore (searcher.py): the observation history
    def get_state(self):
        return {"X": [x.tolist() for x in self.X], "y": list(self.y)}

    def set_state(self, state):
        self.X = [np.asarray(x) for x in state["X"]]
        self.y = list(state["y"])


def _merge(space, point):
    cfg = copy.deepcopy(space)
    for k, v in point.items():
        if isinstance(v, dict) and isinstance(cfg.get(k), dict):
            cfg[k] = _merge(cfg[k], v)
        else:
            cfg[k] = v
    return cfg


class TPESearch(_ModelSearcher):
    """Tree-structured Parzen Estimator.

    Observations are split at the ``gamma`` quantile (at most 25 good points, as Optuna)
    into good/bad sets; each dimension gets a truncated-Gaussian Parzen density over the unit interval plus a uniform prior
    component (categoricals: smoothed frequency tables).  ``n_candidates`` draws from the
    good density are ranked by l(x)/g(x) and the best one is suggested.  The first
    ``n_initial_points`` suggestions are uniform random.
    """

    def __init__(self, space=None, metric=None, mode=None, points_to_evaluate=None,
                 n_initial_points=10, gamma=0.1, n_candidates=24, prior_weight=1.0,
                 seed=None, random_state_seed=None):
        super().__init__(space, metric, mode, points_to_evaluate,
                         seed if seed is not None else random_state_seed)
        self.n_initial_points = n_initial_points
        self.gamma = gamma
        self.n_candidates = n_candidates
        self.prior_weight = prior_weight

    def _propose(self):
        n = len(self.y)
        if n < max(self.n_initial_points, 2):
            return self._random()
        X = np.stack(self.X)
        order = np.argsort(np.asarray(self.y))
        n_good = min(max(1, int(math.ceil(self.gamma * n))), 25)
        good, bad = X[order[:n_good]], X[order[n_good:]]
        sp = self._space
        dims = len(sp.params)
        cands = np.empty((self.n_candidates, dims))
        score = np.zeros(self.n_candidates)
        for d in range(dims):
            if sp.is_numeric(d):
                cands[:, d] = self._sample_parzen(good[:, d])
                score += self._log_parzen(cands[:, d], good[:, d])
                score -= self._log_parzen(cands[:, d], bad[:, d])
            else:
                k = sp.n_choices(d)
                pg = self._cat_probs(good[:, d], k)
                pb = self._cat_probs(bad[:, d], k)
                cands[:, d] = self._rng.choice(k, size=self.n_candidates, p=pg)
                idx = cands[:, d].astype(int)
                score += np.log(pg[idx]) - np.log(pb[idx])
        return cands[int(np.argmax(score))]

    @staticmethod
    def _bandwidth(obs):
        n = len(obs) + 1  # +1 for the uniform prior component
        sd = np.std(obs) if len(obs) > 1 else 0.5
        # Scott's rule, floored like Optuna's "magic clip" (~range / min(100, n)) so the good
        # density never collapses onto the incumbent
        return min(max(1.06 * sd * n ** (-0.2), 0.35 / min(100, n)), 1.0)

    def _sample_parzen(self, obs):
        bw = self._bandwidth(obs)
        m = len(obs)
        w = np.append(np.ones(m), self.prior_weight)
        comp = self._rng.choice(m + 1, size=self.n_candidates, p=w / w.sum())
        out = np.empty(self.n_candidates)
        for j, c in enumerate(comp):
            if c == m:
                out[j] = self._rng.uniform()
                continue
            for _ in range(16):
                v = self._rng.normal(obs[c], bw)
                if 0.0 <= v <= 1.0:
                    break
            out[j] = min(max(v, 0.0), 1.0)
        return out

    def _log_parzen(self, x, obs):
        m = len(obs)
        if m == 0:
            return np.zeros_like(x)
        bw = self._bandwidth(obs)
        z = (x[:, None] - obs[None, :]) / bw
        dens = np.exp(-0.5 * z * z) / (bw * math.sqrt(2 * math.pi))
        total = dens.sum(1) + self.prior_weight   # uniform prior density is 1 on [0, 1]
        return np.log(total / (m + self.prior_weight) + 1e-300)

    def _cat_probs(self, obs, k):
        counts = np.bincount(obs.astype(int), minlength=k).astype(np.float64) + \
            self.prior_weight / k
        return counts / counts.sum()


class BayesOptSearch(_ModelSearcher):
    """Gaussian-process Bayesian optimisation over a continuous box.

    A Matern-5/2 GP (unit-cube inputs, standardised targets, fixed noise) is refit after every
    completed trial; the acquisition (``ucb`` with ``kappa``, ``ei`` or ``poi`` with ``xi``)
    is maximised over random candidates plus Gaussian perturbations of the incumbent.
    Categorical parameters are rejected, as in the reference adapter.
    """

    def __init__(self, space=None, metric=None, mode=None, points_to_evaluate=None,
                 utility_kwargs=None, random_state=None, random_search_steps=10,
                 length_scale=0.25, noise=1e-4, n_candidates=2048):
        super().__init__(space, metric, mode, points_to_evaluate, random_state)
        self.utility = {"kind": "ucb", "kappa": 2.576, "xi": 0.0, **(utility_kwargs or {})}
        self.random_search_steps = random_search_steps
        self.length_scale = length_scale
        self.noise = noise
        self.n_candidates = n_candidates
        if self._space is not None:
            self._check()

    def set_search_properties(self, metric, mode, config):
        super().set_search_properties(metric, mode, config)
        if self._space is not None:
            self._check()
        return True

    def _check(self):
        for path, dom in self._space.params:
            if isinstance(dom, Categorical):
                raise ValueError(f"BayesOptSearch only supports numeric parameters; "
                                 f"{'/'.join(map(str, path))} is categorical")

    def _kernel(self, A, B):
        d = np.sqrt(np.maximum(((A[:, None, :] - B[None, :, :]) ** 2).sum(-1), 0.0)) / \
            self.length_scale
        s5 = math.sqrt(5.0) * d
        return (1.0 + s5 + 5.0 / 3.0 * d * d) * np.exp(-s5)

    def posterior(self, Xs):
        """GP posterior mean/std (internal minimisation sign) at ``Xs``."""
        X = np.stack(self.X)
        y = np.asarray(self.y)
        mu0, sd0 = y.mean(), y.std() + 1e-12
        yn = (y - mu0) / sd0
        K = self._kernel(X, X) + (self.noise + 1e-10) * np.eye(len(X))
        L = np.linalg.cholesky(K)
        alpha = np.linalg.solve(L.T, np.linalg.solve(L, yn))
        Ks = self._kernel(Xs, X)
        v = np.linalg.solve(L, Ks.T)
        var = np.maximum(1.0 - (v * v).sum(0), 1e-12)
        return (Ks @ alpha) * sd0 + mu0, np.sqrt(var) * sd0

    def _propose(self):
        if len(self.y) < max(self.random_search_steps, 2):
            return self._random()
        dims = len(self._space.params)
        best = self.X[int(np.argmin(self.y))]
        cands = np.concatenate([
            self._rng.uniform(size=(self.n_candidates, dims)),
            np.clip(best + self._rng.normal(0, 0.05, size=(self.n_candidates // 4, dims)), 0, 1),
        ])
        mu, sd = self.posterior(cands)
        # maximise the acquisition of f = -y (the internal objective is minimised)
        f, fbest = -mu, -min(self.y)
        kind = self.utility["kind"]
        if kind == "ucb":
            acq = f + self.utility["kappa"] * sd
        else:
            from scipy.stats import norm
            imp = f - fbest - self.utility["xi"]
            z = imp / sd
            acq = imp * norm.cdf(z) + sd * norm.pdf(z) if kind == "ei" else norm.cdf(z)
        return cands[int(np.argmax(acq))]


# reference adapter names (python/ray/tune/search/{hyperopt,optuna}/): both libraries default
# to TPE, which is what these run.
HyperOptSearch = TPESearch
OptunaSearch = TPESearch
