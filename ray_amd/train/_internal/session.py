"""Per-worker training session (reference: python/ray/train/_internal/session.py,
python/ray/train/context.py).

The user's ``train_loop_per_worker`` runs in a thread inside a Train worker
actor. ``train.report`` hands (metrics, checkpoint) to the driver through a
bounded queue that the driver drains with ``get_next`` — the training thread
blocks until the driver has consumed the previous report, keeping all ranks in
lock-step like the reference."""

from __future__ import annotations

import os
import queue
import shutil
import threading
import time
from dataclasses import dataclass, field

from ray_amd.train._checkpoint import Checkpoint


@dataclass
class TrainContext:
    world_rank: int = 0
    local_rank: int = 0
    world_size: int = 1
    local_world_size: int = 1
    node_rank: int = 0
    experiment_name: str = ""
    trial_name: str = ""
    trial_id: str = ""
    trial_dir: str = ""
    storage_path: str = ""
    metadata: dict = field(default_factory=dict)
    # non-local run storage (train/_internal/storage.py): checkpoints are uploaded to
    # ``remote_trial_dir`` on ``storage_filesystem``
    storage_filesystem: object = None
    remote_trial_dir: str = ""

    def get_world_rank(self):
        return self.world_rank

    def get_local_rank(self):
        return self.local_rank

    def get_world_size(self):
        return self.world_size

    def get_local_world_size(self):
        return self.local_world_size

    def get_node_rank(self):
        return self.node_rank

    def get_experiment_name(self):
        return self.experiment_name

    def get_trial_name(self):
        return self.trial_name

    def get_trial_id(self):
        return self.trial_id

    def get_trial_dir(self):
        return self.trial_dir

    def get_storage(self):
        return self.storage_path

    def get_metadata(self):
        return self.metadata


class _Session:
    def __init__(self, ctx: TrainContext, checkpoint: Checkpoint | None, dataset_shards: dict,
                 config: dict, checkpoint_index: int = 0):
        self.ctx = ctx
        self.loaded_checkpoint = checkpoint
        self.dataset_shards = dataset_shards or {}
        self.config = config
        self.results: queue.Queue = queue.Queue(maxsize=1)
        self.continue_ev = threading.Semaphore(0)
        self.finished = False
        self.error = None
        self.thread = None
        self.checkpoint_index = checkpoint_index
        self.iteration = 0
        self.start_time = time.time()

    def report(self, metrics: dict, checkpoint: Checkpoint | None = None):
        self.iteration += 1
        persisted = None
        if checkpoint is not None:
            persisted = self._persist(checkpoint)
        m = dict(metrics)
        m.setdefault("training_iteration", self.iteration)
        m.setdefault("time_total_s", time.time() - self.start_time)
        self.results.put(("report", m, persisted))
        self.continue_ev.acquire()

    def _persist(self, ckpt: Checkpoint) -> str:
        """Copy the worker-local checkpoint dir into the run's storage (all ranks write
        into the same indexed directory, like the reference)."""
        fs = self.ctx.storage_filesystem
        if fs is not None:
            from ray_amd.train._internal import storage

            dst = storage.join(self.ctx.remote_trial_dir,
                               f"checkpoint_{self.checkpoint_index:06d}")
            storage.upload_dir(ckpt.path, fs, dst)
            self.checkpoint_index += 1
            return dst
        dst = os.path.join(self.ctx.trial_dir, f"checkpoint_{self.checkpoint_index:06d}")
        os.makedirs(dst, exist_ok=True)
        if os.path.abspath(ckpt.path) != os.path.abspath(dst):
            shutil.copytree(ckpt.path, dst, dirs_exist_ok=True)
        self.checkpoint_index += 1
        return dst


_session: _Session | None = None


def _get_session(required=True) -> _Session | None:
    if _session is None and required:
        from ray_amd.train.error import SessionMisuseError

        raise SessionMisuseError("`train.report` / `train.get_context` must be called from "
                                 "inside a training function run by a ray_amd Trainer.")
    return _session


def init_session(s: _Session):
    global _session
    _session = s


def shutdown_session():
    global _session
    _session = None


def report(metrics: dict, *, checkpoint: Checkpoint | None = None) -> None:
    s = _get_session(required=False)
    if s is None:
        # Tune function trainables share this entry point
        from ray_amd.tune.trainable import function_report

        return function_report(metrics, checkpoint)
    s.report(metrics, checkpoint)


def get_checkpoint() -> Checkpoint | None:
    s = _get_session(required=False)
    if s is None:
        from ray_amd.tune.trainable import function_get_checkpoint

        return function_get_checkpoint()
    return s.loaded_checkpoint


def get_context() -> TrainContext:
    s = _get_session(required=False)
    if s is None:
        from ray_amd.tune.trainable import function_get_context

        return function_get_context()
    return s.ctx


def get_dataset_shard(name: str = "train"):
    s = _get_session()
    shard = s.dataset_shards.get(name)
    if shard is None:
        raise KeyError(f"no dataset named {name!r} was passed to the Trainer")
    return shard
