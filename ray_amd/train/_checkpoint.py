"""Directory-backed checkpoints (reference: python/ray/train/_checkpoint.py)."""

from __future__ import annotations

import contextlib
import json
import os
import shutil
import tempfile
import uuid

_METADATA = ".metadata.json"


class Checkpoint:
    def __init__(self, path: str, filesystem=None):
        self.path = os.fspath(path)
        self.filesystem = filesystem

    @classmethod
    def from_directory(cls, path) -> "Checkpoint":
        return cls(os.path.abspath(os.fspath(path)))

    @classmethod
    def from_dict(cls, data: dict) -> "Checkpoint":
        import pickle

        d = tempfile.mkdtemp(prefix="ra_ckpt_")
        with open(os.path.join(d, "dict_checkpoint.pkl"), "wb") as f:
            pickle.dump(data, f)
        return cls(d)

    def to_dict(self) -> dict:
        import pickle

        with open(os.path.join(self.path, "dict_checkpoint.pkl"), "rb") as f:
            return pickle.load(f)

    def to_directory(self, path: str | None = None) -> str:
        path = path or os.path.join(tempfile.gettempdir(), f"checkpoint_{uuid.uuid4().hex}")
        os.makedirs(path, exist_ok=True)
        shutil.copytree(self.path, path, dirs_exist_ok=True)
        return path

    @contextlib.contextmanager
    def as_directory(self):
        yield self.path

    def get_metadata(self) -> dict:
        p = os.path.join(self.path, _METADATA)
        if not os.path.exists(p):
            return {}
        with open(p) as f:
            return json.load(f)

    def set_metadata(self, metadata: dict) -> None:
        with open(os.path.join(self.path, _METADATA), "w") as f:
            json.dump(metadata, f)

    def update_metadata(self, metadata: dict) -> None:
        m = self.get_metadata()
        m.update(metadata)
        self.set_metadata(m)

    # framework checkpoints (TorchCheckpoint, SklearnCheckpoint) keep the fitted
    # preprocessor beside the model so a Predictor built from the checkpoint applies it
    # (reference: train/_internal/framework_checkpoint.py)
    PREPROCESSOR_FILENAME = "preprocessor.pkl"

    def set_preprocessor(self, preprocessor) -> None:
        import cloudpickle

        with open(os.path.join(self.path, self.PREPROCESSOR_FILENAME), "wb") as f:
            cloudpickle.dump(preprocessor, f)

    def get_preprocessor(self):
        import pickle

        p = os.path.join(self.path, self.PREPROCESSOR_FILENAME)
        if not os.path.exists(p):
            return None
        with open(p, "rb") as f:
            return pickle.load(f)

    def __repr__(self):
        return f"Checkpoint(filesystem=local, path={self.path})"

    def __eq__(self, o):
        return isinstance(o, Checkpoint) and o.path == self.path

    def __hash__(self):
        return hash(self.path)
