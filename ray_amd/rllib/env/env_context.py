"""``EnvContext`` (reference: python/ray/rllib/env/env_context.py): the ``env_config`` dict
an env creator receives, plus where the env runs — ``worker_index`` (0 = local runner),
``num_workers``, ``vector_index`` (the env's slot in its runner's vector), ``remote``."""

from __future__ import annotations

from typing import Optional


class EnvContext(dict):
    def __init__(self, env_config: Optional[dict] = None, worker_index: int = 0,
                 vector_index: int = 0, remote: bool = False,
                 num_workers: Optional[int] = None, recreated_worker: bool = False):
        super().__init__(env_config or {})
        self.worker_index = int(worker_index)
        self.vector_index = int(vector_index)
        self.remote = bool(remote)
        self.num_workers = num_workers
        self.recreated_worker = recreated_worker

    def copy_with_overrides(self, env_config=None, worker_index=None, vector_index=None,
                            remote=None, num_workers=None, recreated_worker=None):
        return EnvContext(
            dict(self) if env_config is None else env_config,
            self.worker_index if worker_index is None else worker_index,
            self.vector_index if vector_index is None else vector_index,
            self.remote if remote is None else remote,
            self.num_workers if num_workers is None else num_workers,
            self.recreated_worker if recreated_worker is None else recreated_worker)

    def set_defaults(self, defaults: dict) -> None:
        for k, v in defaults.items():
            self.setdefault(k, v)

    def __reduce__(self):
        return (EnvContext, (dict(self), self.worker_index, self.vector_index, self.remote,
                             self.num_workers, self.recreated_worker))

    def __str__(self):
        return (f"EnvContext({dict(self)}, worker_index={self.worker_index}, "
                f"vector_index={self.vector_index})")
