"""Directory-backed checkpoints (reference: python/ray/train/_checkpoint.py).

A checkpoint is a directory on the local filesystem, or on a pyarrow filesystem when
``filesystem`` is given (runs with ``RunConfig.storage_filesystem`` / a URI storage path,
see ``train/_internal/storage.py``). Remote checkpoints are downloaded once, on first
access, into a local temporary directory (``as_directory`` / ``to_directory``)."""

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
        from ray_amd.train._internal.storage import _is_local

        self.path = os.fspath(path)
        self.filesystem = None if _is_local(filesystem) else filesystem
        self._local = None  # download of a remote checkpoint

    def _local_path(self) -> str:
        if self.filesystem is None:
            return self.path
        if getattr(self, "_local", None) is None or not os.path.isdir(self._local):
            from ray_amd.train._internal.storage import download_dir

            d = tempfile.mkdtemp(prefix="ra_ckpt_dl_")
            download_dir(self.filesystem, self.path, d)
            self._local = d
        return self._local

    def __getstate__(self):
        st = dict(self.__dict__)
        st["_local"] = None
        return st

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

        with open(os.path.join(self._local_path(), "dict_checkpoint.pkl"), "rb") as f:
            return pickle.load(f)

    def to_directory(self, path: str | None = None) -> str:
        path = path or os.path.join(tempfile.gettempdir(), f"checkpoint_{uuid.uuid4().hex}")
        os.makedirs(path, exist_ok=True)
        if self.filesystem is not None:
            from ray_amd.train._internal.storage import download_dir

            download_dir(self.filesystem, self.path, path)
        else:
            shutil.copytree(self.path, path, dirs_exist_ok=True)
        return path

    @contextlib.contextmanager
    def as_directory(self):
        yield self._local_path()

    def get_metadata(self) -> dict:
        if self.filesystem is not None:
            from ray_amd.train._internal.storage import join, read_text

            t = read_text(self.filesystem, join(self.path, _METADATA))
            return json.loads(t) if t else {}
        p = os.path.join(self.path, _METADATA)
        if not os.path.exists(p):
            return {}
        with open(p) as f:
            return json.load(f)

    def set_metadata(self, metadata: dict) -> None:
        if self.filesystem is not None:
            from ray_amd.train._internal.storage import join, write_text

            write_text(self.filesystem, join(self.path, _METADATA), json.dumps(metadata))
            self._local = None
            return
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

        if self.filesystem is not None:
            from ray_amd.train._internal.storage import join

            with self.filesystem.open_output_stream(
                    join(self.path, self.PREPROCESSOR_FILENAME)) as f:
                f.write(cloudpickle.dumps(preprocessor))
            self._local = None
            return
        with open(os.path.join(self.path, self.PREPROCESSOR_FILENAME), "wb") as f:
            cloudpickle.dump(preprocessor, f)

    def get_preprocessor(self):
        import pickle

        p = os.path.join(self._local_path(), self.PREPROCESSOR_FILENAME)
        if not os.path.exists(p):
            return None
        with open(p, "rb") as f:
            return pickle.load(f)

    def __repr__(self):
        fs = "local" if self.filesystem is None else self.filesystem.type_name
        return f"{type(self).__name__}(filesystem={fs}, path={self.path})"

    def __eq__(self, o):
        return isinstance(o, Checkpoint) and o.path == self.path

    def __hash__(self):
        return hash(self.path)
