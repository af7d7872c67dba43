"""Offline data for the offline algorithms (BC, MARWIL, CQL) over ray_amd.data
(reference: rllib/offline/offline_data.py — the new stack's ``OfflineData`` over
``ray.data`` — and the old stack's rllib/offline/dataset_reader.py:70,179).

``OfflineData`` reads recorded experience as a Dataset of transition rows
(``io.read_offline_dataset``), adds the per-episode discounted return-to-go MARWIL
weights its advantages by (a ``groupby("eps_id").map_groups`` pass — episodes are
independent, so the groups run as parallel Data tasks), and feeds the learners:

* one local learner: ``sample(n)`` draws from an endless stream of epochs, each a
  ``iter_batches`` pass with a local shuffle buffer;
* N learner actors: ``shards(N)`` is ``streaming_split(N, equal=True)`` — every learner
  pulls its own batches from one coordinated streaming execution, and all shards hold the
  same row count, so the learners run the same number of updates (their gradients meet in
  an all-reduce per update: ``LearnerGroup.update_from_iterator``).
"""

from __future__ import annotations

import numpy as np

from .io import read_offline_dataset


def _returns_of_group(gamma):
    def fn(g):
        order = np.argsort(g["t"], kind="stable")
        g = {k: v[order] for k, v in g.items()}
        r = g["rewards"].astype(np.float64)
        out = np.zeros(len(r), np.float32)
        run = 0.0
        for t in range(len(r) - 1, -1, -1):
            run = r[t] + gamma * run
            out[t] = run
        g["returns"] = out
        return g

    return fn


def add_returns(ds, gamma: float):
    """Discounted return-to-go per row, computed over whole episodes (eps_id groups)."""
    return ds.groupby("eps_id").map_groups(_returns_of_group(float(gamma)))


class OfflineData:
    """Recorded experience for offline training. ``inp``: directory / file / glob / list
    (fragment JSON or transition Parquet). ``read_method`` forces "read_json" or
    "read_parquet"."""

    def __init__(self, inp, gamma: float = 0.99, seed=None, *, read_method=None,
                 read_kwargs=None, shuffle_buffer_size: int | None = None):
        ds = read_offline_dataset(inp, read_method=read_method, read_kwargs=read_kwargs)
        # materialised once: the groupby is an all-to-all, and every epoch re-reads blocks
        self.dataset = add_returns(ds, gamma).materialize()
        self.size = self.dataset.count()
        if self.size == 0:
            raise ValueError(f"offline input {inp!r} holds no transitions")
        self.seed = seed
        self.shuffle_buffer_size = shuffle_buffer_size
        self._gen = None
        self._epoch = 0

    def __len__(self):
        return self.size

    def _buffer(self, n):
        return self.shuffle_buffer_size or max(4 * n, min(self.size, 50_000))

    def _epochs(self, n):
        while True:
            seed = None if self.seed is None else int(self.seed) + self._epoch
            self._epoch += 1
            got = False
            for b in self.dataset.iter_batches(batch_size=n, drop_last=True,
                                               local_shuffle_buffer_size=self._buffer(n),
                                               local_shuffle_seed=seed):
                got = True
                yield b
            if not got:  # fewer rows than one batch: sample with replacement
                rng = np.random.default_rng(seed)
                allb = next(iter(self.dataset.iter_batches(batch_size=self.size)))
                idx = rng.integers(0, self.size, size=n)
                yield {k: v[idx] for k, v in allb.items()}

    def sample(self, n: int) -> dict:
        """The next ``n`` rows of the shuffled epoch stream (a new epoch starts when one
        ends)."""
        if self._gen is None or self._gen_n != n:
            self._gen, self._gen_n = self._epochs(n), n
        return next(self._gen)

    def shards(self, n: int) -> list:
        """``n`` equal streaming shards (one per learner actor)."""
        return self.dataset.streaming_split(n, equal=True)


def iterate_forever(it, batch_size: int, seed=None, shuffle_buffer_size=None):
    """Endless batches from a DataIterator shard: epoch after epoch, each with a local
    shuffle buffer (learner-side consumer of ``OfflineData.shards``)."""
    ep = 0
    while True:
        got = False
        for b in it.iter_batches(batch_size=batch_size, drop_last=True,
                                 local_shuffle_buffer_size=shuffle_buffer_size or
                                 4 * batch_size,
                                 local_shuffle_seed=None if seed is None else seed + ep):
            got = True
            yield b
        ep += 1
        if not got:
            raise ValueError(f"a learner's data shard holds fewer than {batch_size} rows")
