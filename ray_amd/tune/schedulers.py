"""Trial schedulers (reference: python/ray/tune/schedulers/{trial_scheduler,async_hyperband,
hyperband,median_stopping_rule,pbt,resource_changing_scheduler}.py)."""

from __future__ import annotations

import copy
import math
import random

import numpy as np


class TrialScheduler:
    CONTINUE = "CONTINUE"
    PAUSE = "PAUSE"
    STOP = "STOP"
    NOOP = "NOOP"

    def __init__(self, metric=None, mode=None):
        self.metric = metric
        self.mode = mode

    def set_search_properties(self, metric, mode):
        self.metric = self.metric or metric
        self.mode = self.mode or mode

    def _score(self, result):
        v = result.get(self.metric)
        if v is None:
            return None
        return v if self.mode == "max" else -v

    def on_trial_add(self, runner, trial):
        pass

    def on_trial_result(self, runner, trial, result):
        return self.CONTINUE

    def on_trial_complete(self, runner, trial, result):
        pass

    def on_trial_error(self, runner, trial):
        pass

    def choose_trial_to_run(self, runner):
        """A trial to start or resume next, or None for the controller's default (the
        first PENDING trial, then a new one from the searcher)."""
        return None

    _supports_buffered_results = True

    @property
    def supports_buffered_results(self) -> bool:
        return self._supports_buffered_results

    def on_trial_remove(self, runner, trial):
        """A trial was removed (stopped) outside the scheduler's decisions."""

    def debug_string(self) -> str:
        return f"Using {type(self).__name__}"

    def save(self, checkpoint_path: str) -> None:
        import cloudpickle

        with open(checkpoint_path, "wb") as f:
            f.write(cloudpickle.dumps(self.__dict__))

    def restore(self, checkpoint_path: str) -> None:
        import cloudpickle

        with open(checkpoint_path, "rb") as f:
            self.__dict__.update(cloudpickle.loads(f.read()))


class FIFOScheduler(TrialScheduler):
    pass


class _AshaBracket:
    """One ASHA bracket: rungs at grace * rf**(k + s), largest first; a trial reaching a rung
    is cut when its score is below the (1 - 1/rf) quantile of the scores already recorded
    there (reference: tune/schedulers/async_hyperband.py _Bracket)."""

    def __init__(self, grace, max_t, rf, s):
        n = int(math.log(max_t / grace) / math.log(rf) - s + 1) if max_t > grace else 0
        self.rf = rf
        self.s = s
        self.rungs = [(grace * rf ** (k + s), {}) for k in reversed(range(max(n, 0)))]

    def on_result(self, trial_id, t, score):
        for milestone, recorded in self.rungs:
            if t < milestone or trial_id in recorded:
                continue
            stop = False
            if recorded:
                cutoff = float(np.nanpercentile(list(recorded.values()), (1 - 1 / self.rf) * 100))
                stop = score < cutoff
            recorded[trial_id] = score
            return stop
        return False


class AsyncHyperBandScheduler(TrialScheduler):
    """ASHA (Li et al. 2018): asynchronous successive halving. ``brackets`` > 1 runs several
    brackets with staggered first rungs (grace * rf**s); a new trial joins bracket s with
    probability proportional to exp(#rungs(s)), as in the reference."""

    def __init__(self, time_attr="training_iteration", metric=None, mode=None, max_t=100,
                 grace_period=1, reduction_factor=4, brackets=1, stop_last_trials=True,
                 seed=None):
        super().__init__(metric, mode)
        if grace_period <= 0 or max_t <= 0 or reduction_factor <= 1 or brackets < 1:
            raise ValueError("need grace_period > 0, max_t > 0, reduction_factor > 1, "
                             "brackets >= 1")
        self.time_attr = time_attr
        self.max_t = max_t
        self.rf = reduction_factor
        self.stop_last_trials = stop_last_trials
        self.brackets = [_AshaBracket(grace_period, max_t, reduction_factor, s)
                         for s in range(brackets)]
        self._rng = np.random.default_rng(seed)
        self._assign = {}  # trial_id -> bracket

    @property
    def rungs(self):
        """Milestone -> recorded scores of the first bracket (diagnostics)."""
        return {m: list(r.values()) for m, r in self.brackets[0].rungs}

    def on_trial_add(self, runner, trial):
        sizes = np.array([len(b.rungs) for b in self.brackets], dtype=np.float64)
        p = np.exp(sizes - sizes.max())
        self._assign[trial.trial_id] = self.brackets[
            int(self._rng.choice(len(self.brackets), p=p / p.sum()))]

    def on_trial_result(self, runner, trial, result):
        t = result.get(self.time_attr, 0)
        if t >= self.max_t and self.stop_last_trials:
            return self.STOP
        s = self._score(result)
        if s is None:
            return self.CONTINUE
        b = self._assign.get(trial.trial_id)
        if b is None:
            self.on_trial_add(runner, trial)
            b = self._assign[trial.trial_id]
        return self.STOP if b.on_result(trial.trial_id, t, s) else self.CONTINUE


ASHAScheduler = AsyncHyperBandScheduler


class _HBBracket:
    """One synchronous HyperBand bracket: n0 trials start with budget r0; when every live
    trial has reached the current milestone, the top 1/eta continue to eta x the budget and
    the rest stop (reference: tune/schedulers/hyperband.py _Bracket)."""

    def __init__(self, n0, r0, max_t, eta, s, time_attr, stop_last):
        self.n = n0
        self.r = r0
        self.max_t = max_t
        self.eta = eta
        self.halves = s
        self.time_attr = time_attr
        self.stop_last = stop_last
        self.live = {}  # trial -> last result (None before the first)
        self.to_unpause = set()
        self.processing = False
        self.progress = 0.0
        self.work = 0.0
        n, r = n0, r0
        for _ in range(s + 1):
            self.work += n * r
            n, r = int(math.ceil(n / eta)), min(r * eta, max_t)

    def t_of(self, result):
        return 0 if result is None else result.get(self.time_attr, 0)

    def filled(self):
        return len(self.live) >= self.n

    def iter_done(self):
        return all(self.t_of(r) >= self.r for r in self.live.values())

    def finished(self):
        return self.stop_last and self.halves == 0 and self.iter_done()

    def keep_going(self, trial):
        if not self.stop_last and self.halves == 0:
            return True
        return self.t_of(self.live.get(trial)) < self.r

    def halve(self, sign):
        self.halves -= 1
        self.n = int(math.ceil(self.n / self.eta))
        self.r = int(min(self.r * self.eta, self.max_t))
        ranked = sorted(self.live, key=lambda tr: sign * self.live[tr].get("_hb_metric", 0))
        return ranked[-self.n:], ranked[:-self.n]

    def completion(self):
        return 1.0 if self.finished() else min(self.progress / max(self.work, 1e-9), 1.0)


class HyperBandScheduler(TrialScheduler):
    """Synchronous HyperBand (Li et al. 2017). Brackets s = s_max..0 (most aggressive first)
    hold n(s) = ceil((s_max+1) / (s+1) * eta**s) trials that start with max_t * eta**-s of
    the time attribute; a trial that reaches its bracket's milestone is PAUSED (checkpointed,
    resources released) until all live trials of the bracket got there, then the top 1/eta
    are unpaused with eta x the budget and the others stop. Reference:
    python/ray/tune/schedulers/hyperband.py:42 (brackets), :239 (_process_bracket)."""

    def __init__(self, time_attr="training_iteration", metric=None, mode=None, max_t=81,
                 reduction_factor=3, stop_last_trials=True):
        super().__init__(metric, mode)
        if reduction_factor <= 1 or max_t <= 0:
            raise ValueError("need reduction_factor > 1 and max_t > 0")
        self.time_attr = time_attr
        self.max_t = max_t
        self.eta = reduction_factor
        self.stop_last = stop_last_trials
        self.s_max = int(round(math.log(max_t) / math.log(reduction_factor)))
        self.bands = [[]]  # iterations, each a list of brackets
        self._next_s = self.s_max
        self._cur = None
        self._info = {}  # trial -> bracket
        self.num_stopped = 0

    def _new_bracket(self):
        while True:
            if self._next_s < 0:
                self.bands.append([])
                self._next_s = self.s_max
            s = self._next_s
            self._next_s -= 1
            r0 = int(self.max_t * self.eta ** (-s))
            if r0 > 0:
                n0 = int(math.ceil((self.s_max + 1) / (s + 1) * self.eta ** s))
                b = _HBBracket(n0, r0, self.max_t, self.eta, s, self.time_attr, self.stop_last)
                self.bands[-1].append(b)
                return b

    def on_trial_add(self, runner, trial):
        if not self.metric or not self.mode:
            raise ValueError("HyperBandScheduler needs metric and mode (pass them to the "
                             "scheduler or to TuneConfig)")
        if self._cur is None or self._cur.filled():
            self._cur = self._new_bracket()
        self._cur.live[trial] = None
        self._info[trial] = self._cur

    def on_trial_result(self, runner, trial, result):
        b = self._info.get(trial)
        if b is None or trial not in b.live:
            return self.CONTINUE
        prev = b.t_of(b.live[trial])
        r = dict(result)
        r["_hb_metric"] = result.get(self.metric, 0)
        b.progress += max(b.t_of(r) - prev, 0)
        b.live[trial] = r
        b.to_unpause.discard(trial)
        if b.keep_going(trial):
            return self.CONTINUE
        return self._process(runner, b, trial)

    def _process(self, runner, b, current=None):
        action = self.PAUSE
        if not b.live or not b.iter_done():
            return action
        if b.finished():
            for tr in list(b.live):
                if tr is not current and tr.status == "PAUSED":
                    runner.stop_trial(tr)
            return self.STOP
        b.processing = True
        sign = 1 if self.mode == "max" else -1
        good, bad = b.halve(sign)
        self.num_stopped += len(bad)
        for tr in bad:
            b.live.pop(tr, None)
            if tr is current:
                action = self.STOP
            elif tr.status == "PAUSED":
                runner.stop_trial(tr)
        for tr in good:
            if b.keep_going(tr):
                if tr is current:
                    action = self.CONTINUE
                else:
                    b.to_unpause.add(tr)
            elif b.finished():
                if tr is current:
                    action = self.STOP
                elif tr.status == "PAUSED":
                    runner.stop_trial(tr)
        b.processing = False
        return action

    def _remove(self, runner, trial):
        b = self._info.get(trial)
        if b is None:
            return
        b.live.pop(trial, None)
        b.to_unpause.discard(trial)
        if not b.processing and b.live and not b.finished():
            self._process(runner, b)

    def on_trial_complete(self, runner, trial, result):
        self._remove(runner, trial)

    def on_trial_error(self, runner, trial):
        self._remove(runner, trial)

    def choose_trial_to_run(self, runner):
        """PENDING trials and unpaused trials, least-complete bracket first."""
        for band in self.bands:
            for b in sorted(band, key=lambda x: x.completion()):
                for tr in b.live:
                    if tr.status == "PENDING" or (tr.status == "PAUSED" and tr in b.to_unpause):
                        return tr
        return None


class MedianStoppingRule(TrialScheduler):
    def __init__(self, time_attr="time_total_s", metric=None, mode=None, grace_period=60.0,
                 min_samples_required=3, min_time_slice=0, hard_stop=True):
        super().__init__(metric, mode)
        self.time_attr = time_attr
        self.grace = grace_period
        self.min_samples = min_samples_required
        self.hist = {}

    def on_trial_result(self, runner, trial, result):
        """Stop a trial whose best score so far is below the median, over the other
        trials (running or finished), of their running mean score up to the same time
        (reference: tune/schedulers/median_stopping_rule.py)."""
        s = self._score(result)
        if s is None:
            return self.CONTINUE
        t = result.get(self.time_attr, 0)
        self.hist.setdefault(trial.trial_id, []).append((t, s))
        if t < self.grace:
            return self.CONTINUE
        others = []
        for k, v in self.hist.items():
            if k == trial.trial_id:
                continue
            upto = [x for tt, x in v if tt <= t]
            if upto:
                others.append(np.mean(upto))
        if len(others) < self.min_samples:
            return self.CONTINUE
        if max(x for _, x in self.hist[trial.trial_id]) < np.median(others):
            return self.STOP
        return self.CONTINUE


class PopulationBasedTraining(TrialScheduler):
    """PBT (Jaderberg et al. 2017): every perturbation_interval, bottom-quantile trials
    clone the checkpoint of a top-quantile trial and perturb its hyperparameters."""

    def __init__(self, time_attr="training_iteration", metric=None, mode=None,
                 perturbation_interval=5, hyperparam_mutations=None, quantile_fraction=0.25,
                 resample_probability=0.25, perturbation_factors=(1.2, 0.8),
                 custom_explore_fn=None, seed=None, log_config=True):
        super().__init__(metric, mode)
        self.log_config = log_config
        self.policy_log = {}  # trial_id -> [(step, new_config)] (PopulationBasedTrainingReplay)
        self.time_attr = time_attr
        self.interval = perturbation_interval
        self.mutations = hyperparam_mutations or {}
        self.q = quantile_fraction
        self.p_resample = resample_probability
        self.factors = perturbation_factors
        self.explore_fn = custom_explore_fn
        self.rng = random.Random(seed)
        self.last = {}
        self.scores = {}
        self.num_perturbations = 0

    def _explore(self, config):
        new = copy.deepcopy(config)
        from ray_amd.tune.search.sample import Domain

        for k, spec in self.mutations.items():
            if isinstance(spec, dict):
                continue
            if self.rng.random() < self.p_resample or k not in new:
                new[k] = spec.sample(self.rng) if isinstance(spec, Domain) else \
                    (self.rng.choice(spec) if isinstance(spec, list) else spec())
            elif isinstance(spec, list):
                i = spec.index(new[k]) if new[k] in spec else 0
                i = max(0, min(len(spec) - 1, i + self.rng.choice([-1, 1])))
                new[k] = spec[i]
            else:
                new[k] = new[k] * self.rng.choice(self.factors)
                if isinstance(config[k], int):
                    new[k] = int(new[k])
        if self.explore_fn:
            new = self.explore_fn(new)
        return new

    def on_trial_result(self, runner, trial, result):
        t = result.get(self.time_attr, 0)
        s = self._score(result)
        if s is None:
            return self.CONTINUE
        self.scores[trial.trial_id] = (s, trial)
        if t - self.last.get(trial.trial_id, 0) < self.interval:
            return self.CONTINUE
        self.last[trial.trial_id] = t
        ranked = sorted(self.scores.values(), key=lambda x: x[0])
        n = len(ranked)
        k = max(1, int(math.ceil(n * self.q))) if n > 1 else 0
        bottom = [tr for _, tr in ranked[:k]]
        top = [tr for _, tr in ranked[-k:]] if k else []
        if trial in top and hasattr(runner, "_save_trial"):
            # a top trial checkpoints at its perturbation interval so bottom trials can
            # clone it (class trainables save on demand; reference: PBT
            # _checkpoint_or_exploit)
            runner._save_trial(trial)
        if trial in bottom and top and trial not in top:
            donor = self.rng.choice(top)
            if donor.last_checkpoint is not None:
                new_cfg = self._explore(donor.config)
                trial.pending_exploit = (donor.last_checkpoint, new_cfg)
                self.num_perturbations += 1
                if self.log_config:
                    self._log_policy(trial, donor, t, new_cfg)
        return self.CONTINUE


    def _log_policy(self, trial, donor, step, new_cfg):
        """Append [trial, donor, step, new_config] to the trial's policy file
        (pbt_policy_<trial_id>.txt in the trial dir) for PopulationBasedTrainingReplay."""
        import json
        import os

        entry = [trial.trial_id, donor.trial_id, int(step), _jsonable(new_cfg)]
        self.policy_log.setdefault(trial.trial_id, []).append(entry)
        d = getattr(trial, "local_path", None)
        if d:
            try:
                os.makedirs(d, exist_ok=True)
                with open(os.path.join(d, f"pbt_policy_{trial.trial_id}.txt"), "a") as f:
                    f.write(json.dumps(entry) + "\n")
            except OSError:
                pass


def _jsonable(cfg):
    out = {}
    for k, v in cfg.items():
        if isinstance(v, dict):
            out[k] = _jsonable(v)
        elif isinstance(v, (int, float, str, bool)) or v is None:
            out[k] = v
        elif hasattr(v, "item"):
            out[k] = v.item()
        else:
            out[k] = repr(v)
    return out


class PopulationBasedTrainingReplay(TrialScheduler):
    """Replays one PBT trial's hyperparameter schedule (reference: tune/schedulers/
    pbt.py PopulationBasedTrainingReplay): the trial starts with the first logged
    config and switches config (keeping its own checkpoint) at each logged step."""

    def __init__(self, policy_file: str):
        import json

        with open(policy_file) as f:
            entries = [json.loads(ln) for ln in f if ln.strip()]
        if not entries:
            raise ValueError(f"{policy_file} holds no PBT policy entries")
        self.schedule = sorted((int(e[2]), e[3]) for e in entries)
        self.config = self.schedule[0][1]
        self._next = 1
        super().__init__()

    def on_trial_add(self, runner, trial):
        trial.config = dict(self.config)

    def on_trial_result(self, runner, trial, result):
        step = result.get("training_iteration", 0)
        if self._next < len(self.schedule) and step >= self.schedule[self._next][0]:
            _, cfg = self.schedule[self._next]
            self._next += 1
            if trial.last_checkpoint is not None:
                trial.pending_exploit = (trial.last_checkpoint, dict(cfg))
        return self.CONTINUE


class PB2(PopulationBasedTraining):
    """Population Based Bandits (Parker-Holder et al. 2020; reference:
    python/ray/tune/schedulers/pb2.py). Exploit like PBT, but explore by GP-UCB instead
    of random perturbation: a Gaussian process (RBF kernel, numpy — no GPy needed) is
    fitted to (time, normalised hyperparameters) -> reward change over the last
    perturbation interval, and the new configuration maximises mu + kappa * sigma over
    random candidates inside ``hyperparam_bounds``."""

    def __init__(self, time_attr="training_iteration", metric=None, mode=None,
                 perturbation_interval=5, hyperparam_bounds=None, quantile_fraction=0.25,
                 log_config=False, require_attrs=True, synch=False, seed=None,
                 kappa=2.0, n_candidates=512):
        super().__init__(time_attr, metric, mode, perturbation_interval, {},
                         quantile_fraction, 0.0, (1.2, 0.8), None, seed)
        self.bounds = {k: (float(v[0]), float(v[1])) for k, v in (hyperparam_bounds or {}).items()}
        self.kappa = kappa
        self.n_cand = n_candidates
        self.np_rng = np.random.default_rng(seed)
        self.data = []  # (t, x_norm..., dy)
        self.prev = {}  # trial_id -> (t, score)

    def _norm(self, cfg):
        return [(float(cfg.get(k, lo)) - lo) / max(hi - lo, 1e-12)
                for k, (lo, hi) in self.bounds.items()]

    def on_trial_result(self, runner, trial, result):
        t = result.get(self.time_attr, 0)
        sc = self._score(result)
        if sc is not None and t - self.last.get(trial.trial_id, 0) >= self.interval:
            pt = self.prev.get(trial.trial_id)
            if pt is not None:
                self.data.append([t] + self._norm(trial.config) + [sc - pt[1]])
                self.data = self.data[-256:]
            self.prev[trial.trial_id] = (t, sc)
        return super().on_trial_result(runner, trial, result)

    @staticmethod
    def _gp(X, y, Xs, ls=0.3, noise=1e-2):
        def k(a, b):
            d = ((a[:, None, :] - b[None, :, :]) ** 2).sum(-1)
            return np.exp(-0.5 * d / ls ** 2)

        K = k(X, X) + noise * np.eye(len(X))
        L = np.linalg.cholesky(K)
        alpha = np.linalg.solve(L.T, np.linalg.solve(L, y))
        Ks = k(Xs, X)
        mu = Ks @ alpha
        v = np.linalg.solve(L, Ks.T)
        var = np.clip(1.0 - (v ** 2).sum(0), 1e-12, None)
        return mu, np.sqrt(var)

    def _explore(self, config):
        new = copy.deepcopy(config)
        if not self.bounds:
            return new
        d = len(self.bounds)
        cand = self.np_rng.random((self.n_cand, d))
        if len(self.data) >= 3:
            D = np.asarray(self.data, np.float64)
            tmax = max(D[:, 0].max(), 1.0)
            X = np.concatenate([D[:, :1] / tmax, D[:, 1:1 + d]], 1)
            y = D[:, -1]
            y = (y - y.mean()) / (y.std() + 1e-8)
            Xs = np.concatenate([np.ones((self.n_cand, 1)), cand], 1)
            mu, sd = self._gp(X, y, Xs)
            best = cand[int(np.argmax(mu + self.kappa * sd))]
        else:
            best = cand[0]  # not enough data yet: uniform sample
        for (k, (lo, hi)), u in zip(self.bounds.items(), best):
            val = lo + float(u) * (hi - lo)
            new[k] = int(round(val)) if isinstance(config.get(k), int) else val
        return new


class HyperBandForBOHB(HyperBandScheduler):
    """HyperBand brackets for BOHB (reference: tune/schedulers/hb_bohb.py). The BOHB
    model-based searcher (hpbandster / ConfigSpace) is not installed; paired with any
    searcher this runs the same early-stopping brackets as HyperBandScheduler."""


def evenly_distribute_cpus_gpus(runner, trial, result, scheduler):
    """Reference DistributeResources: split the cluster's CPUs/GPUs evenly over the live
    trials (never below the trial's base request)."""
    import ray_amd as ray

    live = [t for t in runner.trials if t.status in ("RUNNING", "PENDING")] or [trial]
    tot = ray.cluster_resources()
    base = scheduler.base_resources.setdefault(trial.trial_id, dict(trial.resources))
    out = dict(base)
    out["CPU"] = max(base.get("CPU", 1), float(int(tot.get("CPU", 1) // len(live))))
    if base.get("GPU"):
        out["GPU"] = max(base["GPU"], float(int(tot.get("GPU", 0) // len(live))))
    return out


DistributeResources = evenly_distribute_cpus_gpus


class ResourceChangingScheduler(TrialScheduler):
    """Re-allocates trial resources while they run (reference:
    python/ray/tune/schedulers/resource_changing_scheduler.py): after each result the
    allocation function proposes resources; a change checkpoints-and-restarts the trial
    with the new request (same config)."""

    def __init__(self, base_scheduler=None, resources_allocation_function=None):
        super().__init__()
        self.base = base_scheduler or FIFOScheduler()
        self.alloc = resources_allocation_function or evenly_distribute_cpus_gpus
        self.base_resources = {}
        self.num_reallocations = 0

    def set_search_properties(self, metric, mode):
        self.base.set_search_properties(metric, mode)

    def on_trial_add(self, runner, trial):
        self.base_resources[trial.trial_id] = dict(trial.resources)
        if hasattr(self.base, "on_trial_add"):
            self.base.on_trial_add(runner, trial)

    def on_trial_complete(self, runner, trial, result):
        self.base.on_trial_complete(runner, trial, result)

    def on_trial_error(self, runner, trial):
        self.base.on_trial_error(runner, trial)

    def choose_trial_to_run(self, runner):
        return self.base.choose_trial_to_run(runner)

    def on_trial_result(self, runner, trial, result):
        decision = self.base.on_trial_result(runner, trial, result)
        if decision != self.CONTINUE or trial.pending_exploit is not None:
            return decision
        new = self.alloc(runner, trial, result, self)
        if new and {k: float(v) for k, v in new.items()} != \
                {k: float(v) for k, v in trial.resources.items()} and \
                trial.last_checkpoint is not None:
            trial.pending_exploit = (trial.last_checkpoint, trial.config)
            trial.pending_resources = dict(new)
            self.num_reallocations += 1
        return decision


_SCHEDULERS = {"fifo": "FIFOScheduler", "async_hyperband": "AsyncHyperBandScheduler",
               "asynchyperband": "AsyncHyperBandScheduler", "asha": "ASHAScheduler",
               "median_stopping_rule": "MedianStoppingRule", "medianstopping": "MedianStoppingRule",
               "hyperband": "HyperBandScheduler", "hb_bohb": "HyperBandForBOHB",
               "pbt": "PopulationBasedTraining", "pbt_replay": "PopulationBasedTrainingReplay",
               "pb2": "PB2", "resource_changing": "ResourceChangingScheduler"}


def create_scheduler(scheduler, **kwargs):
    """A trial scheduler by name (reference: tune/schedulers/__init__.py
    create_scheduler); an instance passes through."""
    if not isinstance(scheduler, str):
        return scheduler
    key = scheduler.lower()
    if key not in _SCHEDULERS:
        raise ValueError(f"Scheduler must be one of {sorted(_SCHEDULERS)}. Got: {scheduler}")
    return globals()[_SCHEDULERS[key]](**kwargs)
