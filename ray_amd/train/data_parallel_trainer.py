"""DataParallelTrainer + BackendExecutor (reference: python/ray/train/
data_parallel_trainer.py, _internal/backend_executor.py, base_trainer.py).

``fit()``: reserve one placement-group bundle per worker, start the worker actors,
run the backend's ``on_start`` (process-group rendezvous), launch the training
loop in every worker and drain reports in lock-step. Rank-0 metrics become the
result; checkpoints are persisted to ``<storage_path>/<name>/checkpoint_XXXXXX``
and pruned to ``CheckpointConfig.num_to_keep`` by score. On a worker failure the
whole group restarts from the latest checkpoint, up to ``FailureConfig.max_failures``
times.
"""

from __future__ import annotations

import json
import os
import shutil
import time
import uuid

import ray_amd as ray
from ray_amd.air.config import CheckpointConfig, RunConfig, ScalingConfig
from ray_amd.train._checkpoint import Checkpoint
from ray_amd.train._internal.session import TrainContext
from ray_amd.train._internal.worker_group import WorkerGroup
from ray_amd.train.backend import BackendConfig
from ray_amd.train.base_trainer import BaseTrainer
from ray_amd.train.result import Result


class TrainingFailedError(RuntimeError):
    pass


class _CheckpointManager:
    def __init__(self, cfg: CheckpointConfig):
        self.cfg = cfg
        self.items: list[tuple[Checkpoint, dict]] = []

    def register(self, ckpt: Checkpoint, metrics: dict):
        """Keep the best ``num_to_keep`` by score (by recency without a score attribute),
        plus always the latest one, which a restore resumes from (reference:
        train/_internal/checkpoint_manager.py register_checkpoint)."""
        self.items.append((ckpt, metrics))
        k = self.cfg.num_to_keep
        if k is None or len(self.items) <= k:
            return
        latest = self.items[-1]
        attr = self.cfg.checkpoint_score_attribute
        if attr:
            rev = self.cfg.checkpoint_score_order == "max"
            missing = float("-inf") if rev else float("inf")
            ranked = sorted(self.items, key=lambda x: x[1].get(attr, missing), reverse=rev)
        else:
            ranked = self.items[::-1]
        drop = [x for x in ranked[k:] if x is not latest]
        for c, _ in drop:
            if c.filesystem is not None:
                from ray_amd.train._internal.storage import delete_dir

                delete_dir(c.filesystem, c.path)
            else:
                shutil.rmtree(c.path, ignore_errors=True)
        self.items = [x for x in self.items if not any(x is d for d in drop)]

    @property
    def latest(self):
        return self.items[-1][0] if self.items else None

    @property
    def best(self):
        attr = self.cfg.checkpoint_score_attribute
        if not self.items:
            return None
        if not attr:
            return self.items[-1][0]
        rev = self.cfg.checkpoint_score_order == "max"
        return sorted(self.items, key=lambda x: x[1].get(attr, 0), reverse=rev)[0][0]


class DataParallelTrainer(BaseTrainer):
    _default_backend_config = BackendConfig

    def __init__(self, train_loop_per_worker, *, train_loop_config: dict | None = None,
                 backend_config: BackendConfig | None = None,
                 scaling_config: ScalingConfig | None = None,
                 run_config: RunConfig | None = None, datasets: dict | None = None,
                 dataset_config=None, resume_from_checkpoint: Checkpoint | None = None,
                 metadata: dict | None = None):
        self.train_loop_per_worker = train_loop_per_worker
        self.train_loop_config = train_loop_config
        self.backend_config = backend_config or self._default_backend_config()
        self.scaling_config = scaling_config or ScalingConfig()
        self.run_config = run_config or RunConfig()
        self.datasets = datasets or {}
        self.dataset_config = dataset_config
        self.resume_from_checkpoint = resume_from_checkpoint
        self.metadata = metadata or {}

    # ---------------------------------------------------------------------------
    def _shards(self, n):
        shards = [dict() for _ in range(n)]
        for name, ds in self.datasets.items():
            cfg = self.dataset_config
            if cfg is None or not hasattr(cfg, "datasets_to_split"):
                from ray_amd.train.data_config import DataConfig

                cfg = DataConfig()
            split = cfg.datasets_to_split == "all" or name in cfg.datasets_to_split
            if split and hasattr(ds, "streaming_split"):
                parts = ds.streaming_split(n, equal=True)
                for i in range(n):
                    shards[i][name] = parts[i]
            else:
                for i in range(n):
                    shards[i][name] = ds.iterator() if hasattr(ds, "iterator") else ds
        return shards

    def fit(self) -> Result:
        from ray_amd.tune.callback import CallbackList
        from ray_amd.tune.logger import default_callbacks

        if not ray.is_initialized():
            ray.init()
        rc = self.run_config
        name = rc.name or f"{type(self).__name__}_{time.strftime('%Y-%m-%d_%H-%M-%S')}"
        from ray_amd.train._internal import storage

        fs, root = storage.resolve(rc.storage_path, rc.storage_filesystem)
        if fs is None:
            trial_dir, remote_dir = os.path.join(root, name), None
        else:  # local staging for the driver's files; checkpoints go straight to fs
            staging = os.environ.get("RAY_AMD_STORAGE", os.path.expanduser("~/ray_amd_results"))
            trial_dir, remote_dir = os.path.join(staging, name), storage.join(root, name)
            fs.create_dir(remote_dir, recursive=True)
        self._storage = (fs, remote_dir)
        os.makedirs(trial_dir, exist_ok=True)
        self._save_trainer(trial_dir)
        mgr = _CheckpointManager(rc.checkpoint_config)
        history = []
        failures = 0
        ckpt = self.resume_from_checkpoint
        ckpt_index = getattr(self, "_restored_ckpt_index", 0)
        error = None
        # RunConfig.callbacks (+ default JSON/CSV loggers) see the run as one trial, the
        # same events a Tuner fires (reference: Trainer.fit runs as a Tune trial)
        trial = _TrainerTrial(name, self.train_loop_config, trial_dir)
        cbs = CallbackList(default_callbacks(rc.callbacks))
        cbs.fire("setup", stop=rc.stop, num_samples=1, total_num_samples=1)
        cbs.fire("on_trial_restore" if ckpt is not None else "on_trial_start", trials=[trial],
                 trial=trial)

        def on_report(metrics, cpath):
            cbs.step([trial])
            trial.last_result = metrics
            cbs.fire("on_trial_result", trials=[trial], trial=trial, result=metrics)
            if cpath:
                cbs.fire("on_trial_save", trials=[trial], trial=trial)
                cbs.fire("on_checkpoint", trials=[trial], trial=trial,
                         checkpoint=Checkpoint(cpath, filesystem=self._storage[0]))
                self._save_state(trial_dir, cpath, metrics)
            cbs.end_step([trial])
            for hook in getattr(self, "_report_hooks", ()):
                hook(metrics, cpath)

        while True:
            try:
                metrics, ckpt_index = self._run_once(trial_dir, name, ckpt, ckpt_index, mgr,
                                                     history, on_report)
                error = None
                break
            except TrainingFailedError as e:
                failures += 1
                error = e
                maxf = rc.failure_config.max_failures
                if maxf != -1 and failures > maxf:
                    break
                cbs.fire("on_trial_recover", trials=[trial], trial=trial)
                ckpt = mgr.latest or ckpt
        if error is not None:
            trial.status = "ERROR"
            cbs.fire("on_trial_error", trials=[trial], trial=trial)
            cbs.fire("on_experiment_end", trials=[trial])
            self._sync_up(trial_dir)
            raise error
        trial.status = "TERMINATED"
        cbs.fire("on_trial_complete", trials=[trial], trial=trial)
        cbs.fire("on_experiment_end", trials=[trial])
        self._sync_up(trial_dir)
        return Result(metrics=history[-1] if history else {}, checkpoint=mgr.latest, error=None,
                      path=remote_dir or trial_dir, metrics_history=history,
                      best_checkpoints=[(c, m) for c, m in mgr.items], filesystem=fs)

    def _sync_up(self, trial_dir):
        """Upload the staged driver files (result.json, progress.csv, trainer state) to a
        non-local run storage."""
        fs, remote_dir = getattr(self, "_storage", (None, None))
        if fs is not None:
            from ray_amd.train._internal import storage

            storage.upload_dir(trial_dir, fs, remote_dir)

    # ------------------------------------------------------------------ restore
    _TRAINER_FILE = "trainer.pkl"
    _STATE_FILE = "trainer_state.json"

    def _save_trainer(self, trial_dir):
        """Persist the trainer definition (minus datasets, which are re-supplied on
        restore) so ``restore(path)`` can rebuild it (reference: base_trainer.py:250)."""
        import cloudpickle

        d = dict(self.__dict__)
        d["_dataset_names"] = list((self.datasets or {}).keys())
        d["datasets"] = {}
        d.pop("resume_from_checkpoint", None)
        try:
            blob = cloudpickle.dumps((type(self), d))
        except Exception:  # noqa: BLE001 - unpicklable user state: restore needs overrides
            return
        tmp = os.path.join(trial_dir, self._TRAINER_FILE + ".tmp")
        with open(tmp, "wb") as f:
            f.write(blob)
        os.replace(tmp, os.path.join(trial_dir, self._TRAINER_FILE))

    def _save_state(self, trial_dir, cpath, metrics):
        st = {"latest_checkpoint": os.path.basename(cpath),
              "metrics": {k: v for k, v in metrics.items()
                          if isinstance(v, (int, float, str, bool))}}
        tmp = os.path.join(trial_dir, self._STATE_FILE + ".tmp")
        with open(tmp, "w") as f:
            json.dump(st, f)
        os.replace(tmp, os.path.join(trial_dir, self._STATE_FILE))

    @classmethod
    def can_restore(cls, path) -> bool:
        return os.path.exists(os.path.join(path, cls._TRAINER_FILE))

    @classmethod
    def restore(cls, path, datasets: dict | None = None, train_loop_per_worker=None,
                train_loop_config: dict | None = None, **overrides):
        """Rebuild an interrupted trainer from its run directory and resume from the latest
        persisted checkpoint. Datasets must be passed again (they are not pickled)."""
        import cloudpickle

        if "://" in str(path):
            raise NotImplementedError(
                "restore() reads a local run directory: download the run from its storage "
                "filesystem first (pyarrow.fs.copy_files)")
        path = os.path.abspath(os.path.expanduser(path))
        with open(os.path.join(path, cls._TRAINER_FILE), "rb") as f:
            tcls, d = cloudpickle.loads(f.read())
        obj = tcls.__new__(tcls)
        obj.__dict__.update(d)
        missing = [n for n in d.get("_dataset_names", []) if n not in (datasets or {})]
        if missing:
            raise ValueError(f"restore() needs the datasets the run was started with: "
                             f"{missing}")
        obj.datasets = datasets or {}
        if train_loop_per_worker is not None:
            obj.train_loop_per_worker = train_loop_per_worker
        if train_loop_config is not None:
            obj.train_loop_config = train_loop_config
        for k, v in overrides.items():
            setattr(obj, k, v)
        import copy

        rc = copy.copy(obj.run_config)
        rc.name = os.path.basename(path)
        rc.storage_path = os.path.dirname(path)
        obj.run_config = rc
        ckpts = sorted(x for x in os.listdir(path) if x.startswith("checkpoint_") and
                       os.path.isdir(os.path.join(path, x)) and os.listdir(os.path.join(path, x)))
        obj.resume_from_checkpoint = Checkpoint(os.path.join(path, ckpts[-1])) if ckpts \
            else None
        obj._restored_ckpt_index = (int(ckpts[-1].split("_")[-1]) + 1) if ckpts else 0
        return obj

    def _run_once(self, trial_dir, name, ckpt, ckpt_index, mgr, history, on_report=None):
        sc = self.scaling_config
        wg = WorkerGroup(sc.num_workers, sc._resources_per_worker_not_none,
                         sc.placement_strategy, trainer_resources=sc._trainer_bundle)
        backend = self.backend_config.backend_cls()
        try:
            try:
                backend.on_start(wg, self.backend_config)
            except Exception as e:
                raise TrainingFailedError(f"backend setup failed: {e!r}") from e
            shards = self._shards(sc.num_workers)
            node_ranks = {}
            local_counts = {}
            futs = []
            trial_id = uuid.uuid4().hex[:8]
            for rank, (w, info) in enumerate(zip(wg.workers, wg.infos)):
                nid = info["node_id"]
                node_ranks.setdefault(nid, len(node_ranks))
                lr = local_counts.get(nid, 0)
                local_counts[nid] = lr + 1
                ctx = TrainContext(world_rank=rank, local_rank=lr, world_size=sc.num_workers,
                                   node_rank=node_ranks[nid], experiment_name=name,
                                   trial_name=name, trial_id=trial_id, trial_dir=trial_dir,
                                   storage_path=self.run_config.storage_path,
                                   metadata=self.metadata,
                                   storage_filesystem=self._storage[0],
                                   remote_trial_dir=self._storage[1] or "")
                futs.append((w, ctx))
            for w, ctx in futs:
                ctx.local_world_size = local_counts[wg.infos[ctx.world_rank]["node_id"]]
            ray.get([w.start_training.remote(self.train_loop_per_worker, self.train_loop_config,
                                             ctx, ckpt, shards[ctx.world_rank], ckpt_index)
                     for w, ctx in futs])
            done = [False] * len(futs)
            while not all(done):
                try:
                    outs = ray.get([w.get_next.remote() for (w, _), d in zip(futs, done)
                                    if not d])
                except ray.exceptions.RayActorError as e:
                    raise TrainingFailedError(f"a training worker died: {e}") from e
                idx = [i for i, d in enumerate(done) if not d]
                rank0 = None
                for i, (kind, a, b) in zip(idx, outs):
                    if kind == "error":
                        exc, tb = a
                        raise TrainingFailedError(f"training function raised on rank {i}:\n{tb}"
                                                  ) from exc
                    if kind == "done":
                        done[i] = True
                    elif i == 0:
                        rank0 = (a, b)
                if rank0 is not None:
                    metrics, cpath = rank0
                    history.append(metrics)
                    if cpath:
                        c = Checkpoint(cpath, filesystem=self._storage[0])
                        mgr.register(c, metrics)
                        ckpt_index = int(os.path.basename(cpath).split("_")[-1]) + 1
                    if on_report is not None:
                        on_report(metrics, cpath)
                    stop = self.run_config.stop
                    if stop and _should_stop(stop, metrics):
                        break
            return (history[-1] if history else {}), ckpt_index
        finally:
            try:
                backend.on_shutdown(wg, self.backend_config)
            except Exception:
                pass
            wg.shutdown()



class _TrainerTrial:
    """The single pseudo-trial a Trainer run presents to Tune callbacks."""

    def __init__(self, name, config, path):
        self.trial_id = name
        self.config = config or {}
        self.local_path = path
        self.path = path
        self.status = "RUNNING"
        self.last_result = {}

    def __repr__(self):
        return f"TrainerTrial({self.trial_id}, {self.status})"


def _should_stop(stop, metrics):
    if callable(stop):
        return stop(metrics)
    for k, v in stop.items():
        if k in metrics and metrics[k] >= v:
            return True
    return False


class TrainingIterator:
    """Iterate a trainer's reports as they arrive (reference: train/trainer.py
    TrainingIterator): ``for metrics in TrainingIterator(trainer): ...``; the final
    ``Result`` is ``it.result`` once exhausted (errors re-raise from the iteration)."""

    def __init__(self, trainer: DataParallelTrainer):
        self._trainer = trainer
        self.result = None

    def __iter__(self):
        import queue
        import threading

        q: queue.Queue = queue.Queue()
        done = object()
        self._trainer._report_hooks = [lambda m, c: q.put(dict(m))]

        def run():
            try:
                self.result = self._trainer.fit()
                q.put(done)
            except BaseException as e:  # noqa: BLE001
                q.put(e)

        th = threading.Thread(target=run, daemon=True, name="TrainingIterator")
        th.start()
        try:
            while True:
                item = q.get()
                if item is done:
                    return
                if isinstance(item, BaseException):
                    raise item
                yield item
        finally:
            th.join(timeout=0.1)
            self._trainer._report_hooks = []
