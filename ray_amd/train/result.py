"""Training result (reference: python/ray/air/result.py)."""

from __future__ import annotations

from dataclasses import dataclass, field


@dataclass
class Result:
    metrics: dict | None
    checkpoint: object = None
    error: BaseException | None = None
    path: str | None = None
    metrics_history: list = field(default_factory=list)
    best_checkpoints: list = field(default_factory=list)
    _config: dict | None = None
    filesystem: object = None  # pyarrow filesystem of ``path`` (None: local)

    @property
    def metrics_dataframe(self):
        import pandas as pd

        return pd.DataFrame(self.metrics_history)

    @property
    def config(self):
        return self._config if self._config is not None else (self.metrics or {}).get("config")

    def get_best_checkpoint(self, metric: str, mode: str = "max"):
        if not self.best_checkpoints:
            return None
        rev = mode == "max"
        return sorted(self.best_checkpoints, key=lambda x: x[1].get(metric, 0), reverse=rev)[0][0]

    @classmethod
    def from_path(cls, path):
        import json
        import os

        hist = []
        p = os.path.join(path, "result.json")
        if os.path.exists(p):
            with open(p) as f:
                hist = [json.loads(x) for x in f if x.strip()]
        ck = sorted(d for d in os.listdir(path) if d.startswith("checkpoint_"))
        from ray_amd.train._checkpoint import Checkpoint

        return cls(metrics=hist[-1] if hist else {}, checkpoint=Checkpoint(os.path.join(path, ck[-1]))
                   if ck else None, path=path, metrics_history=hist)
