"""``RandomAccessDataset`` (reference: python/ray/data/random_access_dataset.py): the dataset
sorted by a key and range-partitioned over actors; ``get_async`` / ``multiget`` route by
partition bounds and binary-search inside the owning actor."""

from __future__ import annotations

from typing import List

import numpy as np

import ray_amd as ray
from ray_amd.data import block as B


class _RAPartition:
    def __init__(self, blk: dict, key: str):
        self.key = key
        self.blk = blk
        self.keys = np.asarray(blk[key]) if blk else np.array([])

    def get(self, k):
        i = int(np.searchsorted(self.keys, k))
        if i < len(self.keys) and self.keys[i] == k:
            return {c: B._py(v[i]) for c, v in self.blk.items()}
        return None

    def multiget(self, ks):
        return [self.get(k) for k in ks]

    def stats(self):
        return {"num_rows": int(len(self.keys))}


class RandomAccessDataset:
    """Key lookups over a dataset sorted by ``key`` and range-partitioned onto
    ``num_workers`` actors (reference: data/random_access_dataset.py)."""

    def __init__(self, ds, key: str, num_workers: int):
        rows = B.concat([ray.get(r) for r in ds.sort(key).get_internal_block_refs()])
        n = B.num_rows(rows) if rows else 0
        num_workers = max(1, min(num_workers, n or 1))
        per = -(-n // num_workers) if n else 0
        Part = ray.remote(num_cpus=0)(_RAPartition)
        self._key = key
        self._actors, self._lo = [], []
        for w in range(num_workers):
            s, e = w * per, min(n, (w + 1) * per)
            if s >= e and w > 0:
                break
            blk = B.slice_block(rows, s, e) if n else {}
            self._actors.append(Part.remote(blk, key))
            self._lo.append(blk[key][0] if n else None)

    def _owner(self, k) -> int:
        if len(self._actors) == 1 or self._lo[0] is None:
            return 0
        return max(0, int(np.searchsorted(np.asarray(self._lo[1:]), k, side="right")))

    def get_async(self, key):
        return self._actors[self._owner(key)].get.remote(key)

    def multiget(self, keys: List) -> List:
        groups: dict = {}
        for i, k in enumerate(keys):
            groups.setdefault(self._owner(k), []).append(i)
        out: list = [None] * len(keys)
        refs = {a: self._actors[a].multiget.remote([keys[i] for i in idx])
                for a, idx in groups.items()}
        for a, idx in groups.items():
            for i, v in zip(idx, ray.get(refs[a])):
                out[i] = v
        return out

    def stats(self) -> str:
        st = ray.get([a.stats.remote() for a in self._actors])
        return f"RandomAccessDataset: {len(st)} workers, rows per worker " \
               f"{[s['num_rows'] for s in st]}"
