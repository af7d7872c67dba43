"""Tuner / TuneConfig / ResultGrid and the trial controller (reference:
python/ray/tune/{tuner,tune_config,result_grid}.py, execution/tune_controller.py,
stopper/*, search/{basic_variant,concurrency_limiter,searcher}.py)."""

from __future__ import annotations

import json
import os
import pickle
import time
import uuid
from dataclasses import dataclass, field

import ray_amd as ray
from ray_amd.air.config import RunConfig
from ray_amd.train._checkpoint import Checkpoint
from ray_amd.train.result import Result
from ray_amd.tune.schedulers import FIFOScheduler, TrialScheduler
from ray_amd.tune.search.sample import generate_variants
from ray_amd.tune.trainable import _TrialActor


# ------------------------------------------------------------------ searchers
class Searcher:
    def __init__(self, metric=None, mode=None):
        self.metric = metric
        self.mode = mode

    def set_search_properties(self, metric, mode, config):
        self.metric = self.metric or metric
        self.mode = self.mode or mode
        return True

    def suggest(self, trial_id):
        raise NotImplementedError

    def on_trial_result(self, trial_id, result):
        pass

    def on_trial_complete(self, trial_id, result=None, error=False):
        pass

    FINISHED = "FINISHED"
    CKPT_FILE_TMPL = "searcher-state-{}.pkl"

    def add_evaluated_point(self, parameters: dict, value: float, error: bool = False,
                            pruned: bool = False, intermediate_values=None) -> None:
        """Tell the searcher about a configuration evaluated outside it (subclasses that
        model the objective override this; the default ignores it)."""

    def add_evaluated_trials(self, trials_or_analysis, metric: str) -> None:
        trials = getattr(trials_or_analysis, "trials", trials_or_analysis)
        for t in trials or []:
            res = getattr(t, "last_result", None) or {}
            if metric in res:
                self.add_evaluated_point(getattr(t, "config", {}), res[metric],
                                         error=getattr(t, "status", "") == "ERROR")

    def set_max_concurrency(self, max_concurrent: int) -> bool:
        return False

    def get_state(self) -> dict:
        return {k: v for k, v in self.__dict__.items() if not k.startswith("__")}

    def set_state(self, state: dict) -> None:
        self.__dict__.update(state)

    def save(self, checkpoint_path: str) -> None:
        import cloudpickle

        with open(checkpoint_path, "wb") as f:
            f.write(cloudpickle.dumps(self.get_state()))

    def restore(self, checkpoint_path: str) -> None:
        """State written by ``save`` of this process's own searcher (a local file this
        framework created, read back as such)."""
        import cloudpickle

        with open(checkpoint_path, "rb") as f:
            self.set_state(cloudpickle.loads(f.read()))

    def save_to_dir(self, checkpoint_dir: str, session_str: str = "default") -> None:
        os.makedirs(checkpoint_dir, exist_ok=True)
        self.save(os.path.join(checkpoint_dir, self.CKPT_FILE_TMPL.format(session_str)))

    def restore_from_dir(self, checkpoint_dir: str) -> None:
        import glob as _glob

        files = sorted(_glob.glob(os.path.join(checkpoint_dir,
                                               self.CKPT_FILE_TMPL.format("*"))))
        if not files:
            raise RuntimeError(f"no searcher checkpoint in {checkpoint_dir}")
        self.restore(files[-1])


class BasicVariantGenerator(Searcher):
    def __init__(self, points_to_evaluate=None, max_concurrent=0, random_state=None):
        super().__init__()
        self.points = list(points_to_evaluate or [])
        self.seed = random_state
        self._it = None

    def _setup(self, space, num_samples):
        self._it = iter(list(self.points) + list(generate_variants(space, num_samples,
                                                                   self.seed)))

    def suggest(self, trial_id):
        try:
            return next(self._it)
        except StopIteration:
            return None


class ConcurrencyLimiter(Searcher):
    def __init__(self, searcher, max_concurrent):
        super().__init__()
        self.searcher = searcher
        self.max_concurrent = max_concurrent
        self.live = set()

    def set_search_properties(self, metric, mode, config):
        return self.searcher.set_search_properties(metric, mode, config)

    def suggest(self, trial_id):
        if len(self.live) >= self.max_concurrent:
            return "PAUSE"
        c = self.searcher.suggest(trial_id)
        if c is not None and c != "PAUSE":
            self.live.add(trial_id)
        return c

    def on_trial_complete(self, trial_id, result=None, error=False):
        self.live.discard(trial_id)
        self.searcher.on_trial_complete(trial_id, result, error)


class Repeater(Searcher):
    def __init__(self, searcher, repeat=1, set_index=True):
        super().__init__()
        self.searcher = searcher
        self.repeat = repeat
        self._cur = None
        self._n = 0

    def suggest(self, trial_id):
        if self._cur is None or self._n >= self.repeat:
            self._cur = self.searcher.suggest(trial_id)
            self._n = 0
        self._n += 1
        return self._cur


def _lookup_metric(result: dict, key: str):
    """result[key], or a nested value by a "/"-separated path ("env_runners/
    episode_return_mean"), as the reference's flattened result dicts allow."""
    if key in result:
        return result[key]
    cur = result
    for part in key.split("/"):
        if not isinstance(cur, dict) or part not in cur:
            return None
        cur = cur[part]
    return cur


# ------------------------------------------------------------------ stoppers
class Stopper:
    def __call__(self, trial_id, result):
        return False

    def stop_all(self):
        return False


class MaximumIterationStopper(Stopper):
    def __init__(self, max_iter):
        self.max_iter = max_iter

    def __call__(self, trial_id, result):
        return result.get("training_iteration", 0) >= self.max_iter


class FunctionStopper(Stopper):
    def __init__(self, fn):
        self.fn = fn

    def __call__(self, trial_id, result):
        return self.fn(trial_id, result)


class NoopStopper(Stopper):
    """Never stops anything (reference: tune/stopper/noop.py)."""


class TrialPlateauStopper(Stopper):
    """Stop a trial once the standard deviation of its last ``num_results`` values of
    ``metric`` is at most ``std``, after ``grace_period`` results; with
    ``metric_threshold`` the plateau must also be at or beyond it (below for
    mode="min", above for mode="max") (reference: tune/stopper/trial_plateau.py)."""

    def __init__(self, metric, std=0.01, num_results=4, grace_period=4, metric_threshold=None,
                 mode=None):
        if metric_threshold is not None and mode not in ("min", "max"):
            raise ValueError("TrialPlateauStopper: metric_threshold needs mode 'min' or 'max'")
        self.metric, self.std, self.n, self.grace = metric, std, num_results, grace_period
        self.threshold, self.mode = metric_threshold, mode
        self.hist = {}

    def __call__(self, trial_id, result):
        import numpy as np

        if self.metric not in result:
            return False
        h = self.hist.setdefault(trial_id, [])
        h.append(float(result[self.metric]))
        if len(h) < max(self.grace, self.n):
            return False
        last = h[-1]
        if self.threshold is not None and (
                (self.mode == "min" and last > self.threshold) or
                (self.mode == "max" and last < self.threshold)):
            return False
        return float(np.std(h[-self.n:])) <= self.std


class ExperimentPlateauStopper(Stopper):
    """Stop the whole experiment when the best ``top`` values of ``metric`` seen so far
    (over all trials) have a standard deviation of at most ``std`` for more than
    ``patience`` consecutive results (reference: tune/stopper/experiment_plateau.py)."""

    def __init__(self, metric, std=0.001, top=10, mode="min", patience=0):
        if mode not in ("min", "max"):
            raise ValueError("ExperimentPlateauStopper: mode must be 'min' or 'max'")
        if patience < 0 or top < 1:
            raise ValueError("ExperimentPlateauStopper: patience >= 0 and top >= 1")
        self.metric, self.std, self.top, self.mode, self.patience = metric, std, top, mode, \
            patience
        self.best = []
        self.iterations = 0

    def __call__(self, trial_id, result):
        import numpy as np

        if self.metric not in result:
            return False
        v = float(result[self.metric])
        self.best.append(v)
        self.best.sort(reverse=self.mode == "max")
        del self.best[self.top:]
        if len(self.best) == self.top and float(np.std(self.best)) <= self.std:
            self.iterations += 1
        else:
            self.iterations = 0
        return False

    def stop_all(self):
        return self.iterations > self.patience


class TimeoutStopper(Stopper):
    def __init__(self, timeout):
        self.deadline = time.time() + (timeout.total_seconds() if hasattr(timeout,
                                                                         "total_seconds")
                                       else timeout)

    def stop_all(self):
        return time.time() > self.deadline


class CombinedStopper(Stopper):
    def __init__(self, *stoppers):
        self.stoppers = stoppers

    def __call__(self, trial_id, result):
        return any(s(trial_id, result) for s in self.stoppers)

    def stop_all(self):
        return any(s.stop_all() for s in self.stoppers)


# ------------------------------------------------------------------ config / results
@dataclass
class TuneConfig:
    metric: str | None = None
    mode: str | None = None
    search_alg: object = None
    scheduler: object = None
    num_samples: int = 1
    max_concurrent_trials: int | None = None
    time_budget_s: float | None = None
    reuse_actors: bool = False
    trial_name_creator: object = None
    trial_dirname_creator: object = None


class Trial:
    def __init__(self, config, trial_id, exp_dir, resources):
        self.config = config
        self.trial_id = trial_id
        self.status = "PENDING"
        self.results = []
        self.last_result = {}
        self.last_checkpoint = None
        self.error = None
        self.actor = None
        self.pending_ref = None
        self.resources = resources
        self.trial_name = f"trial_{trial_id}"
        self.local_path = os.path.join(exp_dir, f"trial_{trial_id}")
        self.pending_exploit = None
        self._asha_rungs = set()
        self.restore_from = None
        self.num_failures = 0
        self.last_checkpoint_iter = 0  # training_iteration of the result with the checkpoint
        self.start_iteration = 0

    # ------------------------------------------------ reference Trial surface
    PENDING, RUNNING, PAUSED, TERMINATED, ERROR = ("PENDING", "RUNNING", "PAUSED",
                                                   "TERMINATED", "ERROR")

    @property
    def path(self):
        return self.local_path

    @property
    def logdir(self):
        return self.local_path

    @property
    def evaluated_params(self) -> dict:
        from ray_amd.tune.utils import flatten_dict

        return flatten_dict(dict(self.config or {}))

    @property
    def experiment_tag(self) -> str:
        return ",".join(f"{k}={v}" for k, v in sorted(self.evaluated_params.items())
                        if isinstance(v, (int, float, str, bool)))

    @property
    def checkpoint(self):
        """The latest persisted checkpoint (``train.Checkpoint``) or None."""
        if not self.last_checkpoint:
            return None
        from ray_amd.train._checkpoint import Checkpoint

        return self.last_checkpoint if isinstance(self.last_checkpoint, Checkpoint) else \
            Checkpoint(self.last_checkpoint)

    def has_checkpoint(self) -> bool:
        return bool(self.last_checkpoint)

    def has_reported_at_least_once(self) -> bool:
        return bool(self.results)

    def is_finished(self) -> bool:
        return self.status in ("TERMINATED", "ERROR")

    @property
    def node_ip(self):
        return self.last_result.get("node_ip")

    @property
    def error_file(self):
        p = os.path.join(self.local_path, "error.txt")
        return p if os.path.exists(p) else None

    def get_error(self):
        """The trial's failure as an exception (or None)."""
        if self.error is None:
            return None
        from ray_amd.tune.error import TuneError

        return self.error if isinstance(self.error, BaseException) else \
            TuneError(str(self.error))

    def should_stop(self, result: dict) -> bool:
        return bool(result.get("done"))

    def metric_analysis(self) -> dict:
        """Per-metric last / min / max / avg over this trial's results."""
        out = {}
        for r in self.results:
            for k, v in r.items():
                if isinstance(v, (int, float)) and not isinstance(v, bool):
                    m = out.setdefault(k, {"max": v, "min": v, "sum": 0.0, "n": 0})
                    m["max"], m["min"] = max(m["max"], v), min(m["min"], v)
                    m["sum"] += v
                    m["n"] += 1
                    m["last"] = v
        return {k: {"max": m["max"], "min": m["min"], "avg": m["sum"] / m["n"],
                    "last": m["last"]} for k, m in out.items()}

    def get_json_state(self) -> str:
        import json as _json

        return _json.dumps({"trial_id": self.trial_id, "status": self.status,
                            "config": self.evaluated_params, "local_path": self.local_path,
                            "num_failures": self.num_failures},
                           default=str)

    def __repr__(self):
        return f"Trial({self.trial_id}, {self.status})"

    def __str__(self):
        return self.trial_name

    def name_with(self, tc, exp_dir):
        """TuneConfig.trial_name_creator / trial_dirname_creator (callables of the Trial)."""
        if tc is not None and tc.trial_name_creator is not None:
            self.trial_name = str(tc.trial_name_creator(self))
        if tc is not None and tc.trial_dirname_creator is not None:
            d = str(tc.trial_dirname_creator(self))
            if os.sep in d or d in ("", ".", ".."):
                raise ValueError(f"trial_dirname_creator returned an invalid name: {d!r}")
            self.local_path = os.path.join(exp_dir, d)
        return self


class ResultGrid:
    def __init__(self, results: list, experiment_path: str, metric=None, mode=None):
        self._results = results
        self.experiment_path = experiment_path
        self._metric = metric
        self._mode = mode

    @property
    def filesystem(self):
        """The pyarrow filesystem the experiment directory lives on (a URI's scheme, or
        the local filesystem)."""
        import pyarrow.fs as pafs

        p = str(self.experiment_path or "")
        if "://" in p:
            return pafs.FileSystem.from_uri(p)[0]
        return pafs.LocalFileSystem()

    def __len__(self):
        return len(self._results)

    def __getitem__(self, i):
        return self._results[i]

    def __iter__(self):
        return iter(self._results)

    @property
    def errors(self):
        return [r.error for r in self._results if r.error is not None]

    @property
    def num_errors(self):
        return len(self.errors)

    @property
    def num_terminated(self):
        return sum(1 for r in self._results if r.error is None)

    def get_best_result(self, metric=None, mode=None, scope="last", filter_nan_and_inf=True):
        metric = metric or self._metric
        mode = mode or self._mode
        if metric is None or mode is None:
            raise ValueError("get_best_result needs metric and mode")
        import math

        best, bv = None, None
        for r in self._results:
            hist = r.metrics_history or [r.metrics or {}]
            vals = [m.get(metric) for m in hist if m.get(metric) is not None]
            if not vals:
                continue
            if scope == "last":
                v = vals[-1]
            elif scope == "avg":
                v = sum(vals) / len(vals)
            else:
                v = max(vals) if mode == "max" else min(vals)
            if filter_nan_and_inf and (math.isnan(v) or math.isinf(v)):
                continue
            if bv is None or (v > bv if mode == "max" else v < bv):
                best, bv = r, v
        if best is None:
            raise RuntimeError(f"no trial reported {metric}")
        return best

    def get_dataframe(self, filter_metric=None, filter_mode=None):
        import pandas as pd

        rows = []
        for r in self._results:
            row = dict(r.metrics or {})
            for k, v in (r._config or {}).items():
                row[f"config/{k}"] = v
            row["logdir"] = r.path
            rows.append(row)
        return pd.DataFrame(rows)


# ------------------------------------------------------------------ controller
class _Controller:
    def __init__(self, trainable, space, tc: TuneConfig, rc: RunConfig, exp_dir, resources):
        self.trainable = trainable
        self.space = space
        self.tc = tc
        self.rc = rc
        self.exp_dir = exp_dir
        self.resources = resources
        self.scheduler: TrialScheduler = tc.scheduler or FIFOScheduler()
        self.scheduler.set_search_properties(tc.metric, tc.mode)
        self.searcher = tc.search_alg or BasicVariantGenerator()
        self.searcher.set_search_properties(tc.metric, tc.mode, space)
        base = self.searcher.searcher if isinstance(self.searcher, ConcurrencyLimiter) else \
            self.searcher
        # reference SearchGenerator (tune/search/search_generator.py): a non-variant searcher
        # is asked for at most num_samples configs
        self._suggest_limit = None
        if isinstance(base, BasicVariantGenerator):
            base._setup(space, tc.num_samples)
        elif tc.num_samples and tc.num_samples > 0:
            self._suggest_limit = tc.num_samples
        self._n_suggested = 0
        self.trials: list[Trial] = []
        self.stopper = self._make_stopper(rc.stop)
        self.exhausted = False
        self.actor_cls = ray.remote(_TrialActor)
        self.start = time.time()
        fc = rc.failure_config
        self.max_failures = fc.max_failures if fc else 0
        ff = fc.fail_fast if fc else False
        self.fail_fast = ff.upper() if isinstance(ff, str) else bool(ff)
        if isinstance(self.fail_fast, str) and self.fail_fast != "RAISE":
            raise ValueError(f"fail_fast must be a bool or 'raise', got {ff!r}")
        if self.fail_fast and self.max_failures != 0:
            # reference tune_controller: a failing trial ends the experiment, so retries
            # would never run
            raise ValueError("max_failures must be 0 if fail_fast is set")
        self._errored = False
        self._actor_cache = []  # (resource key, actor) for TuneConfig.reuse_actors
        self.num_actor_reuses = 0
        from ray_amd.tune.callback import CallbackList
        from ray_amd.tune.logger import default_callbacks

        # RunConfig.callbacks + the default JSON / CSV loggers (result.json, progress.csv)
        self.cb = CallbackList(default_callbacks(rc.callbacks))
        self.cb.fire("setup", stop=rc.stop, num_samples=tc.num_samples,
                     total_num_samples=tc.num_samples)

    @staticmethod
    def _make_stopper(stop):
        if stop is None:
            return None
        if isinstance(stop, Stopper):
            return stop
        if callable(stop):
            return FunctionStopper(stop)

        class _Dict(Stopper):
            def __call__(self, tid, result):
                for k, v in stop.items():
                    got = _lookup_metric(result, k)
                    if got is not None and got == got and got >= v:  # (NaN never stops)
                        return True
                return False

        return _Dict()

    def _max_concurrent(self):
        cpus = ray.cluster_resources().get("CPU", 1)
        need = max(self.resources.get("CPU", 1), 1e-3)
        gpus = ray.cluster_resources().get("GPU", 0)
        n = int(cpus // need)
        if self.resources.get("GPU"):
            n = min(n, int(gpus // self.resources["GPU"]))
        if self.tc.max_concurrent_trials:
            n = min(n, self.tc.max_concurrent_trials)
        return max(1, n)

    def _new_trial(self):
        if self.exhausted:
            return None
        if self._suggest_limit is not None and self._n_suggested >= self._suggest_limit:
            self.exhausted = True
            return None
        tid = uuid.uuid4().hex[:8]
        cfg = self.searcher.suggest(tid)
        if cfg == "PAUSE":
            return None
        if cfg is None:
            self.exhausted = True
            return None
        self._n_suggested += 1
        t = Trial(cfg, tid, self.exp_dir, self.resources).name_with(self.tc, self.exp_dir)
        self.trials.append(t)
        self.scheduler.on_trial_add(self, t)
        return t

    @staticmethod
    def _res_key(res):
        return tuple(sorted((k, float(v)) for k, v in (res or {}).items()))

    def _log_files(self, actor, t):
        """RunConfig.log_to_file: True -> trial_dir/stdout + stderr; a str -> both streams
        into that file; a (stdout, stderr) pair. Relative names are in the trial dir."""
        spec = getattr(self.rc, "log_to_file", False)
        if not spec:
            return
        if spec is True:
            names = ("stdout", "stderr")
        elif isinstance(spec, str):
            names = (spec, spec)
        elif isinstance(spec, (tuple, list)) and len(spec) == 2:
            names = tuple(spec)
        else:
            raise ValueError("RunConfig.log_to_file must be a bool, a str or a (str, str) pair")
        paths = [n if os.path.isabs(n) else os.path.join(t.local_path, n) for n in names]
        actor.set_log_files.remote(*paths)

    def _launch(self, t: Trial, checkpoint=None):
        res = t.resources or self.resources
        cc = self.rc.checkpoint_config
        t.status = "RUNNING"
        actor = None
        if self.tc.reuse_actors:
            key = self._res_key(res)
            for i, (k, a) in enumerate(self._actor_cache):
                if k == key:
                    self._actor_cache.pop(i)
                    try:
                        ok = ray.get(a.reset.remote(t.config, t.local_path, t.trial_id,
                                                    t.trial_name, checkpoint,
                                                    t.start_iteration), timeout=60)
                    except Exception:  # noqa: BLE001
                        ok = False
                    if ok:
                        actor = a
                        self.num_actor_reuses += 1
                        self._log_files(actor, t)
                    else:
                        ray.kill(a)
                    break
        if actor is None:
            opts = {"num_cpus": res.get("CPU", 1)}
            if res.get("GPU"):
                opts["num_gpus"] = res["GPU"]
            extra = {k: v for k, v in res.items() if k not in ("CPU", "GPU")}
            if extra:
                opts["resources"] = extra
            actor = self.actor_cls.options(**opts).remote(
                self.trainable, t.config, t.local_path, t.trial_id, t.trial_name,
                checkpoint, cc.checkpoint_frequency if cc else 0, t.start_iteration)
            self._log_files(actor, t)
            actor.start.remote()  # actor calls are ordered: next_result runs after start
        t.actor = actor
        t.pending_ref = t.actor.next_result.remote()
        self.cb.fire("on_trial_restore" if checkpoint else "on_trial_start",
                     trials=self.trials, trial=t)

    def _release_actor(self, t, reuse=False):
        if t.actor is None:
            return
        a, t.actor = t.actor, None
        t.pending_ref = None
        try:
            ray.get(a.stop.remote(), timeout=5)
        except Exception:  # noqa: BLE001
            reuse = False
        more = not self.exhausted or any(x.status == "PENDING" for x in self.trials)
        if reuse and self.tc.reuse_actors and more:
            self._actor_cache.append((self._res_key(t.resources or self.resources), a))
        else:
            ray.kill(a)

    def stop_trial(self, t):
        """Scheduler hook (HyperBand): stop a trial that is not the one being processed."""
        if t.status in ("TERMINATED", "ERROR"):
            return
        self._stop_trial(t)

    def _pause_trial(self, t):
        """Scheduler PAUSE: checkpoint the trial (class trainables save on demand; function
        trainables keep the checkpoint of their last report), release its actor, and
        resume it from that checkpoint when the scheduler picks it again. A trial with no
        checkpoint restarts from scratch (as in the reference)."""
        path = self._save_trial(t) if t.actor is not None else None
        if path:
            t.last_checkpoint_iter = t.last_result.get("training_iteration",
                                                       t.last_checkpoint_iter)
        self._release_actor(t, reuse=True)
        t.status = "PAUSED"
        t.restore_from = t.last_checkpoint
        t.start_iteration = t.last_checkpoint_iter if t.last_checkpoint else 0

    def _on_failure(self, t, exc):
        """A trial raised or its actor died: retry from the last checkpoint while
        num_failures <= FailureConfig.max_failures (-1: always), else ERROR; fail_fast ends
        the experiment at the first ERROR, fail_fast='raise' re-raises (reference:
        tune_controller._process_trial_failure, trial.should_recover)."""
        if self.fail_fast == "RAISE":
            for x in self.trials:
                if x.status == "RUNNING" and x is not t:
                    self._stop_trial(x)
            self._release_actor(t)
            raise exc
        t.num_failures += 1
        if self.max_failures < 0 or t.num_failures <= self.max_failures:
            self._release_actor(t)
            t.status = "PENDING"
            t.restore_from = t.last_checkpoint
            t.start_iteration = t.last_checkpoint_iter if t.last_checkpoint else 0
            t.results = [r for r in t.results
                         if r.get("training_iteration", 0) <= t.start_iteration]
            t.last_result = t.results[-1] if t.results else {}
            t.error = None
            self.cb.fire("on_trial_recover", trials=self.trials, trial=t)
            return
        self._stop_trial(t, "ERROR", exc)
        self._errored = True

    def _stop_trial(self, t, status="TERMINATED", error=None):
        t.status = status
        t.error = error
        cc = self.rc.checkpoint_config
        if status == "TERMINATED" and t.actor is not None and cc and cc.checkpoint_at_end:
            try:  # class trainables: one last checkpoint of the finished trial
                path = ray.get(t.actor.save.remote(), timeout=120)
                if path:
                    t.last_checkpoint = path
                    self._log_checkpoint(t, path)
            except Exception:  # noqa: BLE001
                pass
        self._release_actor(t, reuse=(status == "TERMINATED"))
        if status == "ERROR":
            self.scheduler.on_trial_error(self, t)
            self.cb.fire("on_trial_error", trials=self.trials, trial=t)
        else:
            self.scheduler.on_trial_complete(self, t, t.last_result)
            if status == "TERMINATED":
                self.cb.fire("on_trial_complete", trials=self.trials, trial=t)
        self.searcher.on_trial_complete(t.trial_id, t.last_result, error is not None)

    def _log(self, t, result, checkpoint=None):
        """Result / checkpoint events to the callbacks (the JSON and CSV loggers write
        result.json, params.json and progress.csv)."""
        self.cb.fire("on_trial_result", trials=self.trials, trial=t, result=result)
        if checkpoint:
            ck = Checkpoint(checkpoint)
            self.cb.fire("on_trial_save", trials=self.trials, trial=t)
            self.cb.fire("on_checkpoint", trials=self.trials, trial=t, checkpoint=ck)

    def _save_trial(self, t):
        """Checkpoint a running class-trainable trial now (between its train() calls)."""
        if t.actor is None:
            return None
        try:
            path = ray.get(t.actor.save.remote(), timeout=120)
        except Exception:  # noqa: BLE001
            return None
        if path:
            t.last_checkpoint = path
            self._log_checkpoint(t, path)
        return path

    def _log_checkpoint(self, t, path):
        ck = Checkpoint(path)
        self.cb.fire("on_trial_save", trials=self.trials, trial=t)
        self.cb.fire("on_checkpoint", trials=self.trials, trial=t, checkpoint=ck)

    def _save_state(self):
        st = {"trials": [(t.trial_id, t.config, t.status, t.last_checkpoint, t.results)
                         for t in self.trials], "exhausted": self.exhausted}
        with open(os.path.join(self.exp_dir, "experiment_state.pkl"), "wb") as f:
            pickle.dump(st, f)
        self._maybe_sync()

    def _maybe_sync(self, force=False):
        """Upload the staged experiment directory to a non-local run storage (RunConfig
        storage_filesystem / URI), at most every SyncConfig.sync_period seconds and at the
        end of the experiment (reference: tune/execution/experiment_state.py syncing)."""
        fs, remote = getattr(self, "storage", (None, None))
        if fs is None:
            return
        sc = self.rc.sync_config
        period = getattr(sc, "sync_period", 300) if sc is not None else 300
        now = time.time()
        if not force and now - getattr(self, "_last_sync", 0.0) < period:
            return
        from ray_amd.train._internal import storage

        storage.upload_dir(self.exp_dir, fs, remote)
        self._last_sync = now

    def _next_to_run(self):
        choose = getattr(self.scheduler, "choose_trial_to_run", None)
        t = choose(self) if choose is not None else None
        if t is not None:
            return t
        for t in self.trials:
            if t.status == "PENDING":
                return t
        return self._new_trial()

    def _reporter(self):
        """RunConfig.progress_reporter, else a CLIReporter unless verbose=0 (reference:
        tune/progress_reporter.py, tune.py _detect_reporter)."""
        if getattr(self, "_rep", False) is not False:
            return self._rep
        rep = self.rc.progress_reporter
        if rep is None and (self.rc.verbose or 0) >= 1:
            from ray_amd.tune.registry import CLIReporter

            rep = CLIReporter(metric=self.tc.metric, mode=self.tc.mode)
        if rep is not None and hasattr(rep, "setup"):
            rep.setup(start_time=time.time(), total_samples=self.tc.num_samples,
                      metric=self.tc.metric, mode=self.tc.mode)
        self._rep = rep
        return rep

    def _report_progress(self, done=False):
        rep = self._reporter()
        if rep is not None and self.trials and rep.should_report(self.trials, done=done):
            rep.report(self.trials, done)

    def run(self):
        maxc = self._max_concurrent()
        budget = self.tc.time_budget_s
        try:
            self._loop(maxc, budget)
        finally:
            for _, a in self._actor_cache:
                ray.kill(a)
            self._actor_cache = []
        for t in self.trials:  # paused trials the scheduler never resumed
            if t.status == "PAUSED":
                t.status = "TERMINATED"
        self._save_state()
        self._report_progress(done=True)
        self.cb.fire("on_experiment_end", trials=self.trials)
        self._maybe_sync(force=True)
        return self.trials

    def _loop(self, maxc, budget):
        while True:
            running = [t for t in self.trials if t.status == "RUNNING"]
            while len(running) < maxc:
                t = self._next_to_run()
                if t is None:
                    break
                if t.status == "PENDING" and t.restore_from is None and t.last_checkpoint \
                        and t.num_failures:
                    t.restore_from = t.last_checkpoint
                self._launch(t, t.restore_from)
                running.append(t)
            if not running:
                break
            self.cb.step(self.trials)
            refs = {t.pending_ref: t for t in running}
            ready, _ = ray.wait(list(refs), num_returns=1, timeout=1.0)
            if budget and time.time() - self.start > budget:
                for t in running:
                    self._stop_trial(t)
                break
            if self.stopper is not None and self.stopper.stop_all():
                for t in running:
                    self._stop_trial(t)
                break
            for r in ready:
                t = refs[r]
                if t.status != "RUNNING" or t.pending_ref is not r:
                    continue  # stopped by a scheduler while this result was in flight
                try:
                    kind, a, b = ray.get(r)
                except Exception as e:  # noqa: BLE001  (actor died)
                    self._on_failure(t, e)
                    continue
                if kind == "done":
                    self._stop_trial(t)
                    continue
                if kind == "error":
                    self._on_failure(t, RuntimeError(a))
                    continue
                result = dict(a)
                result["trial_id"] = t.trial_id
                result["config"] = t.config
                if b:
                    t.last_checkpoint = b
                    t.last_checkpoint_iter = result.get("training_iteration", 0)
                t.results.append(result)
                t.last_result = result
                self._log(t, result, b)
                self.searcher.on_trial_result(t.trial_id, result)
                decision = self.scheduler.on_trial_result(self, t, result)
                if self.stopper is not None and self.stopper(t.trial_id, result):
                    decision = TrialScheduler.STOP
                if decision == TrialScheduler.STOP:
                    self._stop_trial(t)
                    continue
                if decision == TrialScheduler.PAUSE:
                    self._pause_trial(t)
                    continue
                if t.pending_exploit is not None:
                    ckpt, cfg = t.pending_exploit
                    t.pending_exploit = None
                    self._stop_trial(t, "PENDING")
                    t.status = "PENDING"
                    t.config = cfg
                    t.restore_from = ckpt
                    t.start_iteration = 0
                    if getattr(t, "pending_resources", None):
                        t.resources = t.pending_resources
                        t.pending_resources = None
                    t._asha_rungs = set()
                    continue
                t.pending_ref = t.actor.next_result.remote()
            self.cb.end_step(self.trials)
            self._save_state()
            self._report_progress()
            if self.fail_fast and self._errored:
                for t in self.trials:
                    if t.status in ("RUNNING", "PAUSED"):
                        self._stop_trial(t)
                    elif t.status == "PENDING":
                        t.status = "TERMINATED"
                self.exhausted = True
                break


def _trainer_to_trainable(trainer):
    """Run a Train trainer as a Tune trial: param_space["train_loop_config"] is merged."""
    import copy

    def fn(config):
        from ray_amd.tune.trainable import function_report

        tr = copy.copy(trainer)
        if hasattr(tr, "train_loop_config"):
            tlc = dict(tr.train_loop_config or {})
            tlc.update(config.get("train_loop_config", {}))
            tr.train_loop_config = tlc
        if "scaling_config" in config:
            tr.scaling_config = config["scaling_config"]
        res = tr.fit()
        for m in res.metrics_history[:-1]:
            function_report(m)
        function_report(res.metrics or {}, res.checkpoint)

    return fn


class Tuner:
    def __init__(self, trainable=None, *, param_space=None, tune_config=None, run_config=None,
                 _restore_path=None):
        from ray_amd.tune.registry import resolve_trainable

        self._resume_config = None
        trainable = resolve_trainable(trainable)
        self.trainable = trainable
        if hasattr(param_space, "to_dict") and hasattr(param_space, "algo_class"):
            param_space = param_space.to_dict()  # an RLlib AlgorithmConfig
        self.param_space = param_space or {}
        self.tune_config = tune_config or TuneConfig()
        self.run_config = run_config or RunConfig()
        self._restore_path = _restore_path

    def fit(self) -> ResultGrid:
        if not ray.is_initialized():
            ray.init()
        rc = self.run_config
        name = rc.name or f"tune_{time.strftime('%Y-%m-%d_%H-%M-%S')}"
        from ray_amd.train._internal import storage

        fs, root = storage.resolve(rc.storage_path, rc.storage_filesystem)
        remote = None
        if self._restore_path:
            exp_dir = self._restore_path
        elif fs is None:
            exp_dir = os.path.join(root, name)
        else:  # staged locally, uploaded to the filesystem (_Controller._maybe_sync)
            staging = os.environ.get("RAY_AMD_STORAGE", os.path.expanduser("~/ray_amd_results"))
            exp_dir, remote = os.path.join(staging, name), storage.join(root, name)
            fs.create_dir(remote, recursive=True)
        os.makedirs(exp_dir, exist_ok=True)
        trainable = self.trainable
        resources = {"CPU": 1}
        from ray_amd.train.base_trainer import BaseTrainer

        if isinstance(trainable, BaseTrainer):
            resources = {"CPU": 0}
            trainable = _trainer_to_trainable(trainable)
        elif getattr(trainable, "_ray_amd_resources", None):
            resources = dict(trainable._ray_amd_resources)
            resources = {("CPU" if k == "cpu" else "GPU" if k == "gpu" else k): v
                         for k, v in resources.items()}
        ctl = _Controller(trainable, self.param_space, self.tune_config, rc, exp_dir, resources)
        ctl.storage = (fs, remote) if remote else (None, None)
        if self._restore_path:
            self._restore_into(ctl)
        trials = ctl.run()
        results = []

        def _remote(p):  # staged path -> its uploaded location
            return storage.join(remote, os.path.relpath(p, exp_dir)) if remote and p else p

        for t in trials:
            ck = None
            if t.last_checkpoint:
                ck = Checkpoint(_remote(t.last_checkpoint), filesystem=fs if remote else None)
            results.append(Result(metrics=t.last_result, checkpoint=ck, error=t.error,
                                  path=_remote(t.local_path), metrics_history=t.results,
                                  _config=t.config, filesystem=fs if remote else None))
        return ResultGrid(results, remote or exp_dir, self.tune_config.metric,
                          self.tune_config.mode)

    def _restore_into(self, ctl):
        p = os.path.join(self._restore_path, "experiment_state.pkl")
        if not os.path.exists(p):
            return
        with open(p, "rb") as f:
            st = pickle.load(f)
        for tid, cfg, status, ckpt, results in st["trials"]:
            t = Trial(cfg, tid, ctl.exp_dir, ctl.resources).name_with(ctl.tc, ctl.exp_dir)
            t.results = results
            t.last_result = results[-1] if results else {}
            t.last_checkpoint = ckpt
            rc = self._resume_config or ResumeConfig()
            kind = rc.finished if status == "TERMINATED" else \
                rc.errored if status == "ERROR" else rc.unfinished
            if kind == ResumeConfig.ResumeType.SKIP:
                t.status = status if status in ("TERMINATED", "ERROR") else "TERMINATED"
            else:
                t.status = "PENDING"
                t.restore_from = ckpt if kind == ResumeConfig.ResumeType.RESUME else None
                if kind == ResumeConfig.ResumeType.RESTART:
                    t.results, t.last_result, t.last_checkpoint = [], {}, None
            ctl.trials.append(t)
        ctl.exhausted = st["exhausted"]

    @classmethod
    def restore(cls, path, trainable=None, *, resume_config=None, resume_unfinished=True,
                resume_errored=False, restart_errored=False, **kw):
        if resume_config is None:
            R = ResumeConfig.ResumeType
            resume_config = ResumeConfig(
                unfinished=R.RESUME if resume_unfinished else R.SKIP,
                errored=R.RESTART if restart_errored else R.RESUME if resume_errored else R.SKIP)
        t = cls(trainable, _restore_path=path, **kw)
        t._resume_config = resume_config
        return t

    @classmethod
    def can_restore(cls, path):
        return os.path.exists(os.path.join(path, "experiment_state.pkl"))

    def get_results(self):
        return self.fit()


class ResumeConfig:
    """What ``Tuner.restore`` does with finished / unfinished / errored trials (reference:
    tune/execution/experiment_state.py ResumeConfig): RESUME from the latest checkpoint,
    RESTART from scratch, or SKIP (keep the recorded outcome)."""

    class ResumeType:
        RESUME = "resume"
        RESTART = "restart"
        SKIP = "skip"

    def __init__(self, finished: str = "skip", unfinished: str = "resume",
                 errored: str = "skip"):
        for v in (finished, unfinished, errored):
            if v not in ("resume", "restart", "skip"):
                raise ValueError(f"invalid ResumeType {v!r}")
        self.finished, self.unfinished, self.errored = finished, unfinished, errored


def run(run_or_experiment, *, config=None, num_samples=1, metric=None, mode=None,
        scheduler=None, search_alg=None, stop=None, resources_per_trial=None, name=None,
        storage_path=None, max_concurrent_trials=None, time_budget_s=None, **kw):
    """Legacy tune.run API (also accepts an Experiment or a registered trainable name)."""
    from ray_amd.tune.registry import Experiment, resolve_trainable

    if isinstance(run_or_experiment, Experiment):
        e = run_or_experiment
        return run(e.run, config=e.config, num_samples=e.num_samples, stop=e.stop,
                   resources_per_trial=e.resources_per_trial, name=e.name,
                   storage_path=e.storage_path, metric=metric, mode=mode, scheduler=scheduler,
                   search_alg=search_alg, max_concurrent_trials=max_concurrent_trials,
                   time_budget_s=time_budget_s)
    from ray_amd.air.config import CheckpointConfig

    attr, order = kw.pop("checkpoint_score_attr", None), "max"
    if attr and attr.startswith("min-"):  # legacy "min-<metric>" form
        attr, order = attr[4:], "min"
    ckpt_cfg = CheckpointConfig(num_to_keep=kw.pop("keep_checkpoints_num", None),
                                checkpoint_frequency=kw.pop("checkpoint_freq", 0) or 0,
                                checkpoint_at_end=kw.pop("checkpoint_at_end", None),
                                checkpoint_score_attribute=attr, checkpoint_score_order=order)
    callbacks = kw.pop("callbacks", None)
    raise_on_failed = kw.pop("raise_on_failed_trial", True)
    # reporting only: progress_reporter / verbose go to RunConfig; sync_config has nothing
    # to sync to (storage_path is a local or shared filesystem path here)
    extra_rc = {k: kw.pop(k) for k in ("progress_reporter", "verbose", "sync_config",
                                       "log_to_file") if k in kw}
    t = resolve_trainable(run_or_experiment)
    if resources_per_trial:
        t = _with_res(t, resources_per_trial)
    tuner = Tuner(t, param_space=config or {},
                  tune_config=TuneConfig(metric=metric, mode=mode, num_samples=num_samples,
                                         scheduler=scheduler, search_alg=search_alg,
                                         max_concurrent_trials=max_concurrent_trials,
                                         time_budget_s=time_budget_s),
                  run_config=RunConfig(name=name, storage_path=storage_path, stop=stop,
                                       checkpoint_config=ckpt_cfg, callbacks=callbacks,
                                       **extra_rc))
    grid = tuner.fit()
    if raise_on_failed and grid.num_errors:
        # reference tune.run: TuneError("Trials did not complete", incomplete_trials)
        from ray_amd.tune import TuneError

        failed = [r for r in grid if r.error is not None]
        raise TuneError(f"Trials did not complete: {len(failed)} of {len(grid)} errored "
                        f"(first: {failed[0].error!r})")
    return ExperimentAnalysis(grid, metric, mode)


def _with_res(t, res):
    from ray_amd.tune.trainable import with_resources

    return with_resources(t, res)


class ExperimentAnalysis:
    def __init__(self, grid: ResultGrid, metric, mode):
        self.grid = grid
        self.default_metric = metric
        self.default_mode = mode
        self.trials = list(grid)

    def get_best_config(self, metric=None, mode=None):
        return self.grid.get_best_result(metric or self.default_metric,
                                         mode or self.default_mode).config

    @property
    def best_config(self):
        return self.get_best_config()

    @property
    def best_result(self):
        return self.grid.get_best_result(self.default_metric, self.default_mode).metrics

    def dataframe(self):
        return self.grid.get_dataframe()

    @property
    def results_df(self):
        return self.grid.get_dataframe()


field  # noqa: B018
