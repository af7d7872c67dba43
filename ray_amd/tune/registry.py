"""Trainable / env registry and the legacy Experiment API.

Reference parity: python/ray/tune/registry.py (register_trainable, register_env,
get_trainable_cls), tune/experiment/experiment.py (Experiment), tune/tune.py
(run_experiments), tune/execution/placement_groups.py (PlacementGroupFactory),
tune/progress_reporter.py (ProgressReporter, CLIReporter), tune/search/__init__.py
(create_searcher) and tune/schedulers/__init__.py (create_scheduler).

Names registered here are resolved by ``Tuner`` / ``tune.run`` when the trainable is a
string; RLlib algorithm names ("PPO", "IMPALA", ...) resolve to their Algorithm classes.
"""

from __future__ import annotations

import sys
import time
from typing import Any, Callable, Dict, List, Optional

_TRAINABLES: Dict[str, Any] = {}


def register_trainable(name: str, trainable, warn: bool = True):
    if not (callable(trainable) or isinstance(trainable, type)):
        raise TypeError(f"{trainable!r} is not a function or Trainable class")
    _TRAINABLES[name] = trainable


def register_env(name: str, env_creator: Callable):
    """Shared with RLlib's env registry (``config.environment(name)``)."""
    from ray_amd.rllib.env.envs import register_env as _reg

    _reg(name, env_creator)


def _rllib_algorithms() -> Dict[str, Any]:
    try:
        from ray_amd.rllib.algorithms.registry import _algos
    except Exception:  # noqa: BLE001
        return {}
    return {name: algo for name, (algo, _) in _algos().items()}


_ALGO_TRAINABLES: Dict[Any, Any] = {}


def algorithm_trainable(algo_cls):
    """Tune class trainable running an RLlib Algorithm (reference: Algorithm IS a
    tune.Trainable): the trial config dict (old- or new-stack keys, ``env`` included) is
    applied onto the algorithm's default AlgorithmConfig; ``step`` is one ``train()``;
    checkpoints are the algorithm's own."""
    if algo_cls in _ALGO_TRAINABLES:
        return _ALGO_TRAINABLES[algo_cls]
    from ray_amd.tune.trainable import Trainable

    class _AlgorithmTrainable(Trainable):
        _algo_cls = algo_cls

        def setup(self, config):
            from ray_amd.rllib.algorithms.registry import get_config_class

            cfg = get_config_class(self._algo_cls)()
            cfg.update_from_dict({k: v for k, v in config.items() if k != "__trial_info__"})
            self.algo = self._algo_cls(cfg)

        def step(self):
            r = dict(self.algo.train())
            r.pop("training_iteration", None)  # the Trainable counts iterations
            return r

        def save_checkpoint(self, checkpoint_dir):
            self.algo.save(checkpoint_dir)
            return checkpoint_dir

        def load_checkpoint(self, checkpoint):
            self.algo.restore(checkpoint)

        def cleanup(self):
            self.algo.stop()

    _AlgorithmTrainable.__name__ = _AlgorithmTrainable.__qualname__ = algo_cls.__name__
    _ALGO_TRAINABLES[algo_cls] = _AlgorithmTrainable
    return _AlgorithmTrainable


def _is_algorithm_cls(t) -> bool:
    try:
        from ray_amd.rllib.algorithms.algorithm import Algorithm
    except Exception:  # noqa: BLE001
        return False
    return isinstance(t, type) and issubclass(t, Algorithm)


def get_trainable_cls(name: str):
    if name in _TRAINABLES:
        return resolve_trainable(_TRAINABLES[name])
    algos = _rllib_algorithms()
    if name in algos:
        return algorithm_trainable(algos[name])
    raise ValueError(f"Unknown trainable {name!r}; registered: "
                     f"{sorted(_TRAINABLES) + sorted(algos)}")


def resolve_trainable(t):
    if isinstance(t, str):
        return get_trainable_cls(t)
    if _is_algorithm_cls(t):
        return algorithm_trainable(t)
    return t


class PlacementGroupFactory:
    """Per-trial bundles: ``PlacementGroupFactory([{"CPU": 1}, {"GPU": 1}] * 2)``. A trial's
    resource request is the bundles' sum (the first bundle is the trainable itself)."""

    def __init__(self, bundles: List[Dict[str, float]], strategy: str = "PACK", **kw):
        if not bundles:
            raise ValueError("at least one bundle is required")
        self.bundles = [dict(b) for b in bundles]
        self.strategy = strategy

    @property
    def head_bundle_is_empty(self) -> bool:
        return not any(self.bundles[0].values())

    def required_resources(self) -> Dict[str, float]:
        out: Dict[str, float] = {}
        for b in self.bundles:
            for k, v in b.items():
                out[k] = out.get(k, 0) + v
        return out

    def __eq__(self, other):
        return isinstance(other, PlacementGroupFactory) and \
            (self.bundles, self.strategy) == (other.bundles, other.strategy)

    def __repr__(self):
        return f"PlacementGroupFactory({self.bundles}, strategy={self.strategy!r})"


class Experiment:
    """Legacy experiment spec (name + run + config + stop + resources + num_samples)."""

    def __init__(self, name: str, run, *, stop=None, config=None, resources_per_trial=None,
                 num_samples: int = 1, storage_path: Optional[str] = None, **kw):
        self.name = name
        self.run = run
        self.stop = stop
        self.config = config or {}
        self.resources_per_trial = resources_per_trial
        self.num_samples = num_samples
        self.storage_path = storage_path
        self.kwargs = kw

    @classmethod
    def from_json(cls, name: str, spec: dict):
        spec = dict(spec)
        run = spec.pop("run")
        return cls(name, run, **spec)

    def spec(self) -> dict:
        return {"run": self.run, "stop": self.stop, "config": self.config,
                "resources_per_trial": self.resources_per_trial,
                "num_samples": self.num_samples}


def run_experiments(experiments, *, scheduler=None, search_alg=None, verbose: int = 2,
                    **kw) -> list:
    """Run one or more Experiments (or {name: spec} dicts) sequentially; returns the trials
    of every experiment (list of Result)."""
    from ray_amd.tune.tuner import run

    if isinstance(experiments, Experiment):
        experiments = [experiments]
    elif isinstance(experiments, dict):
        experiments = [Experiment.from_json(n, s) for n, s in experiments.items()]
    trials = []
    for e in experiments:
        ana = run(e.run, config=e.config, num_samples=e.num_samples, stop=e.stop,
                  resources_per_trial=e.resources_per_trial, name=e.name,
                  storage_path=e.storage_path, scheduler=scheduler, search_alg=search_alg,
                  **{**e.kwargs, **kw})
        trials.extend(ana.trials)
    return trials


# ----------------------------------------------------------------------- reporters
class ProgressReporter:
    """Interface: ``should_report(trials, done)`` and ``report(trials, done)``."""

    def setup(self, start_time=None, total_samples=None, metric=None, mode=None, **kw):
        self._start = start_time or time.time()
        self._total = total_samples
        self._metric, self._mode = metric, mode

    def should_report(self, trials, done: bool = False) -> bool:
        return True

    def report(self, trials, done: bool, *sys_info):
        raise NotImplementedError


class CLIReporter(ProgressReporter):
    """Table of trial status / config / latest metrics, printed at most every
    ``max_report_frequency`` seconds (and once when done)."""

    def __init__(self, metric_columns=None, parameter_columns=None, max_report_frequency=5,
                 max_progress_rows=20, sort_by_metric=False, metric=None, mode=None,
                 print_intermediate_tables=None, file=None):
        self.metric_columns = metric_columns
        self.parameter_columns = parameter_columns
        self.max_report_frequency = max_report_frequency
        self.max_progress_rows = max_progress_rows
        self._metric, self._mode = metric, mode
        self._last = 0.0
        self._file = file
        self._start = time.time()

    def add_metric_column(self, metric: str, representation: Optional[str] = None):
        cols = self.metric_columns
        if cols is None:
            self.metric_columns = cols = []
        if isinstance(cols, dict):
            cols[metric] = representation or metric
        else:
            cols.append(metric)

    def should_report(self, trials, done: bool = False) -> bool:
        now = time.time()
        if done or now - self._last >= self.max_report_frequency:
            self._last = now
            return True
        return False

    def _row(self, t) -> List[str]:
        cfg = getattr(t, "config", {}) or {}
        res = getattr(t, "last_result", None) or {}
        pcols = self.parameter_columns or sorted(k for k, v in cfg.items()
                                                  if isinstance(v, (int, float, str)))
        mcols = list(self.metric_columns or [k for k in ("training_iteration", self._metric)
                                             if k])
        return ([str(getattr(t, "trial_id", "?")), str(getattr(t, "status", "?"))]
                + [str(cfg.get(c, "")) for c in pcols] + [str(res.get(c, "")) for c in mcols])

    def report(self, trials, done: bool, *sys_info):
        from tabulate import tabulate

        rows = [self._row(t) for t in list(trials)[: self.max_progress_rows]]
        if not rows:
            return
        cfg0 = getattr(trials[0], "config", {}) or {}
        pcols = self.parameter_columns or sorted(k for k, v in cfg0.items()
                                                  if isinstance(v, (int, float, str)))
        mcols = list(self.metric_columns or [k for k in ("training_iteration", self._metric)
                                             if k])
        out = self._file or sys.stdout
        status = "done" if done else "running"
        print(f"== Status ({status}, {time.time() - self._start:.1f}s) ==", file=out)
        print(tabulate(rows, headers=["trial", "status", *pcols, *mcols]), file=out, flush=True)


class JupyterNotebookReporter(CLIReporter):
    """Same table (no HTML widgets in this build)."""


def create_searcher(search_alg: str, **kwargs):
    from ray_amd.tune import search as S

    table = {"variant_generator": S.BasicVariantGenerator, "random": S.BasicVariantGenerator,
             "hyperopt": S.HyperOptSearch, "optuna": S.OptunaSearch, "tpe": S.TPESearch,
             "bayesopt": S.BayesOptSearch}
    if search_alg not in table:
        raise ValueError(f"Search alg must be one of {sorted(table)}, got {search_alg!r}")
    return table[search_alg](**kwargs)


def create_scheduler(scheduler: str, **kwargs):
    from ray_amd.tune import schedulers as Sc

    table = {"fifo": Sc.FIFOScheduler, "async_hyperband": Sc.AsyncHyperBandScheduler,
             "asynchyperband": Sc.AsyncHyperBandScheduler, "asha": Sc.ASHAScheduler,
             "median_stopping_rule": Sc.MedianStoppingRule, "medianstopping": Sc.MedianStoppingRule,
             "hyperband": Sc.HyperBandScheduler, "hb_bohb": Sc.HyperBandForBOHB,
             "pbt": Sc.PopulationBasedTraining, "pbt_replay": Sc.PopulationBasedTrainingReplay,
             "pb2": Sc.PB2, "resource_changing": Sc.ResourceChangingScheduler}
    if scheduler not in table:
        raise ValueError(f"Scheduler must be one of {sorted(table)}, got {scheduler!r}")
    return table[scheduler](**kwargs)
