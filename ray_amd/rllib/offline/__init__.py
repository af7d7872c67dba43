"""Offline experience I/O (reference: rllib/offline/json_writer.py, json_reader.py,
offline_data.py, and rllib/evaluation/postprocessing.py for MARWIL's returns).

EnvRunners write every sampled fragment when ``config.offline_data(output=dir)`` is
set: one JSON line per fragment, columns as nested lists with a ``"shape"`` header
so [T, B, ...] fragments round-trip exactly. ``OfflineData`` loads a directory (or
glob / list of files) once into flat column arrays — time-major fragments are
unrolled per environment so discounted returns can be computed episode-correctly —
and serves uniformly sampled minibatches to the offline learners (BC, MARWIL, CQL).
"""

from __future__ import annotations

import glob
import json
import os

import numpy as np

_COLS = ("obs", "actions", "rewards", "terminateds", "truncateds", "next_obs",
         "action_logp")


class JsonWriter:
    def __init__(self, path: str, worker_index: int = 0):
        os.makedirs(path, exist_ok=True)
        self.file = os.path.join(path, f"output-worker{worker_index}-{os.getpid()}.json")

    def write(self, batch: dict):
        rec = {}
        for k in _COLS:
            if k in batch:
                v = np.asarray(batch[k])
                rec[k] = {"dtype": str(v.dtype), "shape": list(v.shape), "data": v.ravel().tolist()}
        with open(self.file, "a") as f:
            f.write(json.dumps(rec) + "\n")


def _files(inp):
    if isinstance(inp, (list, tuple)):
        out = []
        for x in inp:
            out += _files(x)
        return out
    if os.path.isdir(inp):
        return sorted(glob.glob(os.path.join(inp, "*.json")))
    return sorted(glob.glob(inp))


class JsonReader:
    def __init__(self, inp):
        self.files = _files(inp)
        if not self.files:
            raise FileNotFoundError(f"no offline data files under {inp!r}")

    def __iter__(self):
        for fn in self.files:
            with open(fn) as f:
                for line in f:
                    line = line.strip()
                    if not line:
                        continue
                    rec = json.loads(line)
                    yield {k: np.asarray(v["data"], dtype=v["dtype"]).reshape(v["shape"])
                           for k, v in rec.items()}


def discounted_returns(rewards, dones, gamma):
    """[T] rewards/dones of one env stream → discounted return-to-go, reset at dones."""
    out = np.zeros(len(rewards), np.float32)
    run = 0.0
    for t in range(len(rewards) - 1, -1, -1):
        if dones[t]:
            run = 0.0
        run = rewards[t] + gamma * run
        out[t] = run
    return out


class OfflineData:
    def __init__(self, inp, gamma: float = 0.99, seed=None):
        cols = {k: [] for k in _COLS}
        rets = []
        for b in JsonReader(inp):
            T, B = b["rewards"].shape[:2]
            done = np.maximum(b["terminateds"], b.get("truncateds", 0 * b["terminateds"]))
            for i in range(B):  # env-major so each stream is contiguous
                for k in _COLS:
                    if k in b:
                        cols[k].append(b[k][:, i])
                rets.append(discounted_returns(b["rewards"][:, i], done[:, i], gamma))
        self.data = {k: np.concatenate(v) for k, v in cols.items() if v}
        self.data["returns"] = np.concatenate(rets)
        self.size = len(self.data["rewards"])
        self.rng = np.random.default_rng(seed)

    def __len__(self):
        return self.size

    def sample(self, n: int) -> dict:
        idx = self.rng.integers(0, self.size, size=n)
        return {k: v[idx] for k, v in self.data.items()}
