"""Old-stack offline I/O interfaces (reference: python/ray/rllib/offline/{io_context,
input_reader,output_writer,mixed_input,shuffled_input}.py).

``IOContext`` tells an input/output factory where it runs; ``InputReader.next()`` yields
batches (``SampleBatch`` dicts); ``OutputWriter.write(batch)`` consumes them. ray_amd's
own offline path reads through ray_amd.data (``read_offline_dataset``); these classes let
reference-style readers and writers plug in (an ``input_`` factory taking an IOContext)."""

from __future__ import annotations

import random
from typing import Any, Dict, Iterator, List, Optional


class IOContext:
    def __init__(self, log_dir: Optional[str] = None, config=None, worker_index: int = 0,
                 worker=None):
        self.log_dir = log_dir or "."
        self.config = config if config is not None else {}
        self.worker_index = worker_index
        self.worker = worker

    def _get(self, key, default=None):
        c = self.config
        return c.get(key, default) if isinstance(c, dict) else getattr(c, key, default)

    @property
    def input_config(self):
        return self._get("input_config", {}) or {}

    @property
    def output_config(self):
        return self._get("output_config", {}) or {}

    def default_sampler_input(self):
        return None


class InputReader:
    """``next()`` -> one batch; iterating yields batches forever."""

    def next(self):
        raise NotImplementedError

    def __iter__(self) -> Iterator[Any]:
        while True:
            yield self.next()


class OutputWriter:
    def write(self, sample_batch) -> None:
        raise NotImplementedError


class NoopOutput(OutputWriter):
    def write(self, sample_batch) -> None:
        pass


class ShuffledInput(InputReader):
    """Shuffles the batches of ``child`` through a buffer of ``n`` batches."""

    def __init__(self, child: InputReader, n: int = 0, seed=None):
        self.child, self.n = child, int(n)
        self.buffer: List[Any] = []
        self._rng = random.Random(seed)

    def next(self):
        if self.n <= 1:
            return self.child.next()
        while len(self.buffer) < self.n:
            self.buffer.append(self.child.next())
        i = self._rng.randrange(len(self.buffer))
        out = self.buffer[i]
        self.buffer[i] = self.child.next()
        return out


class MixedInput(InputReader):
    """Draws each batch from one of several inputs with the given probabilities:
    ``{"sampler": 0.4, "/data/a": 0.3, reader_or_factory: 0.3}``; path keys read with
    ``JsonReader``."""

    def __init__(self, dist: Dict[Any, float], ioctx: IOContext = None, seed=None):
        total = sum(dist.values())
        if abs(total - 1.0) > 1e-6:
            raise ValueError(f"MixedInput probabilities must sum to 1, got {total}")
        self._rng = random.Random(seed)
        self.choices, self.p = [], []
        for k, v in dist.items():
            if isinstance(k, InputReader):
                src = k
            elif callable(k):
                src = k(ioctx)
            elif k == "sampler":
                src = ioctx.default_sampler_input() if ioctx is not None else None
                if src is None:
                    raise ValueError("MixedInput 'sampler' needs an IOContext with a sampler")
            else:
                from ray_amd.rllib.offline.io import JsonReader

                src = _IterInput(JsonReader(k))
            self.choices.append(src)
            self.p.append(v)

    def next(self):
        return self._rng.choices(self.choices, weights=self.p)[0].next()


class _IterInput(InputReader):
    def __init__(self, it):
        self._src = it
        self._it = iter(it)

    def next(self):
        try:
            return next(self._it)
        except StopIteration:
            self._it = iter(self._src)
            return next(self._it)


class DatasetReader(InputReader):
    """Batches of ``batch_size`` rows from a ray_amd.data Dataset (reference:
    offline/dataset_reader.py), cycling over the data."""

    def __init__(self, ds, ioctx: IOContext = None, batch_size: Optional[int] = None):
        self.ds = ds
        self.batch_size = batch_size or (ioctx._get("train_batch_size", 1) if ioctx else 1)
        self._it = None

    def next(self):
        from ray_amd.rllib.policy_sample_batch import SampleBatch

        for _ in range(2):
            if self._it is None:
                self._it = iter(self.ds.iter_batches(batch_size=self.batch_size,
                                                     batch_format="numpy"))
            try:
                return SampleBatch(next(self._it))
            except StopIteration:
                self._it = None
        raise ValueError("the dataset is empty")


class DatasetWriter(OutputWriter):
    """Buffers batches and writes them as JSON or Parquet shards (reference:
    offline/dataset_writer.py) through ray_amd.data, every ``max_num_samples_per_file``
    rows and on ``flush``."""

    def __init__(self, ioctx: IOContext = None, compress_columns=None, path: str = None,
                 format: str = "json", max_num_samples_per_file: int = 100_000):
        self.path = path or (ioctx.output_config.get("path") if ioctx else None) or \
            (ioctx.log_dir if ioctx else ".")
        self.format = (ioctx.output_config.get("format") if ioctx else None) or format
        self.max_rows = int((ioctx.output_config.get("max_num_samples_per_file")
                             if ioctx else None) or max_num_samples_per_file)
        self.worker_index = ioctx.worker_index if ioctx else 0
        self._rows: List[dict] = []
        self._n = 0

    def write(self, sample_batch) -> None:
        import numpy as np

        cols = {k: np.asarray(v) for k, v in dict(sample_batch).items()}
        n = len(next(iter(cols.values()))) if cols else 0
        for i in range(n):
            self._rows.append({k: v[i] for k, v in cols.items()})
        if len(self._rows) >= self.max_rows:
            self.flush()

    def flush(self) -> None:
        if not self._rows:
            return
        from ray_amd import data as rd

        ds = rd.from_items(self._rows)
        sub = f"{self.path}/w{self.worker_index}_{self._n:05d}"
        (ds.write_parquet if self.format == "parquet" else ds.write_json)(sub)
        self._n += 1
        self._rows = []


def get_dataset_and_shards(config, num_workers: int = 0):
    """(dataset, [per-runner shards]) of an ``input_`` path (reference:
    offline/dataset_reader.get_dataset_and_shards)."""
    from ray_amd.rllib.offline.io import read_offline_dataset

    inp = config.get("input_") if isinstance(config, dict) else config.input_
    ds = read_offline_dataset(inp)
    if num_workers <= 0:
        return ds, [ds]
    return ds, [None] + ds.split(num_workers)


def get_offline_io_resource_bundles(config) -> List[Dict[str, float]]:
    """Resources of the read tasks of an offline dataset input: ray_amd reads in the
    cluster's ordinary task slots, so none are reserved."""
    return []
