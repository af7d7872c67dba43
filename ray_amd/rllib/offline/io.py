"""Offline experience I/O (reference: rllib/offline/json_writer.py, json_reader.py,
dataset_writer.py, dataset_reader.py:70,179).

Two on-disk forms:

* **Fragment JSON** (``output_write_method="write_json"``, the default): EnvRunners append
  one JSON line per sampled [T, B] fragment, columns as flat lists with a ``shape``
  header so fragments round-trip exactly.
* **Transition Parquet** (``output_write_method="write_parquet"``): one row per env step
  with ``eps_id`` / ``t`` columns and tensor observations as fixed-size lists — the
  schema every reader below produces, readable by any Parquet tool.

``read_offline_dataset`` turns either form (or a list / glob of files) into a
``ray_amd.data`` Dataset of transition rows: obs, actions, rewards, terminateds,
truncateds, next_obs, action_logp, action_prob (when recorded), eps_id, t. Fragment files
are decoded by ``FragmentJsonDatasource``, one read task per file, so a runner's env
streams stay contiguous and every episode gets one id.
"""

from __future__ import annotations

import glob
import json
import os

import numpy as np

_COLS = ("obs", "actions", "rewards", "terminateds", "truncateds", "next_obs",
         "action_logp")


class JsonWriter:
    """One JSON line per sampled fragment (reference: json_writer.py)."""

    def __init__(self, path: str, worker_index: int = 0):
        os.makedirs(path, exist_ok=True)
        self.file = os.path.join(path, f"output-worker{worker_index}-{os.getpid()}.json")

    def write(self, batch: dict):
        rec = {}
        for k in _COLS + ("loss_mask",):
            if k in batch:
                v = np.asarray(batch[k])
                rec[k] = {"dtype": str(v.dtype), "shape": list(v.shape),
                          "data": v.ravel().tolist()}
        with open(self.file, "a") as f:
            f.write(json.dumps(rec) + "\n")


class ParquetWriter:
    """Transition rows into Parquet files (reference: dataset_writer.py). Every ``write``
    unrolls a [T, B] fragment env-major into rows with stable episode ids; a file is
    closed every ``max_rows_per_file`` rows."""

    def __init__(self, path: str, worker_index: int = 0, max_rows_per_file: int = 100_000):
        os.makedirs(path, exist_ok=True)
        self.path, self.worker_index = path, worker_index
        self.max_rows = int(max_rows_per_file)
        self._rows, self._nfile = [], 0
        self._streams = _Streams(worker_index * 1_000_003 + os.getpid() % 1000)

    def write(self, batch: dict):
        blk = fragment_to_transitions(batch, self._streams)
        if not len(blk["rewards"]):
            return
        self._rows.append(blk)
        if sum(len(b["rewards"]) for b in self._rows) >= self.max_rows:
            self.flush()

    def flush(self):
        if not self._rows:
            return
        import pyarrow.parquet as pq

        from ray_amd.data import block as B

        blk = {k: np.concatenate([b[k] for b in self._rows]) for k in self._rows[0]}
        fn = os.path.join(self.path, f"output-worker{self.worker_index}-{os.getpid()}-"
                                     f"{self._nfile:05d}.parquet")
        pq.write_table(B.to_batch(blk, "pyarrow"), fn)
        self._nfile += 1
        self._rows = []

    def __del__(self):
        try:
            self.flush()
        except Exception:  # noqa: BLE001
            pass


def _files(inp, exts=(".json",)):
    if isinstance(inp, (list, tuple)):
        out = []
        for x in inp:
            out += _files(x, exts)
        return out
    if os.path.isdir(inp):
        return sorted(f for e in exts for f in glob.glob(os.path.join(inp, f"*{e}")))
    return sorted(glob.glob(inp))


class JsonReader:
    """Iterate the recorded fragments of fragment-JSON files (reference: json_reader.py)."""

    def __init__(self, inp):
        self.files = _files(inp)
        if not self.files:
            raise FileNotFoundError(f"no offline data files under {inp!r}")

    def __iter__(self):
        for fn in self.files:
            yield from read_fragments(fn)


def read_fragments(fn):
    with open(fn) as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            rec = json.loads(line)
            yield {k: np.asarray(v["data"], dtype=v["dtype"]).reshape(v["shape"])
                   for k, v in rec.items()}


class _Streams:
    """Episode ids of the env streams of one writer / file: column i of consecutive
    fragments is the same env, so an episode cut by a fragment boundary keeps its id."""

    def __init__(self, base: int):
        self.base = int(base) << 20
        self.next_id = 0
        self.cur: dict[int, tuple[int, int]] = {}  # column -> (eps_id, t)

    def start(self, col):
        if col not in self.cur:
            self.cur[col] = (self.base + self.next_id, 0)
            self.next_id += 1
        return self.cur[col]

    def advance(self, col, done):
        eid, t = self.cur[col]
        if done:
            del self.cur[col]
        else:
            self.cur[col] = (eid, t + 1)


def fragment_to_transitions(b: dict, streams: _Streams) -> dict:
    """A [T, B] fragment -> transition rows (env-major; padding rows of complete-episode
    fragments dropped) with eps_id / t and action_prob = exp(action_logp)."""
    T, Bn = b["rewards"].shape[:2]
    done = np.maximum(b["terminateds"], b.get("truncateds", np.zeros_like(b["terminateds"])))
    mask = b.get("loss_mask")
    nxt = b.get("next_obs")
    if nxt is None:  # rolled forward within the fragment; the last row repeats
        nxt = np.concatenate([b["obs"][1:], b["obs"][-1:]], 0)
    cols = {k: [] for k in ("obs", "actions", "rewards", "terminateds", "truncateds",
                            "next_obs", "eps_id", "t")}
    has_lp = "action_logp" in b
    if has_lp:
        cols["action_logp"] = []
    for i in range(Bn):
        rows = np.arange(T) if mask is None else np.nonzero(mask[:, i] > 0)[0]
        if not len(rows):
            continue
        eids = np.empty(len(rows), np.int64)
        ts = np.empty(len(rows), np.int64)
        for j, t in enumerate(rows):
            eids[j], ts[j] = streams.start(i)
            streams.advance(i, bool(done[t, i]))
        cols["obs"].append(b["obs"][rows, i])
        cols["actions"].append(b["actions"][rows, i])
        cols["rewards"].append(b["rewards"][rows, i].astype(np.float32))
        cols["terminateds"].append(b["terminateds"][rows, i].astype(np.float32))
        tr = b.get("truncateds")
        cols["truncateds"].append((tr[rows, i] if tr is not None
                                   else np.zeros(len(rows))).astype(np.float32))
        cols["next_obs"].append(nxt[rows, i])
        cols["eps_id"].append(eids)
        cols["t"].append(ts)
        if has_lp:
            cols["action_logp"].append(b["action_logp"][rows, i].astype(np.float32))
    if not cols["rewards"]:
        return {"rewards": np.zeros(0, np.float32)}
    out = {k: np.concatenate(v) for k, v in cols.items()}
    if has_lp:
        out["action_prob"] = np.exp(out["action_logp"]).astype(np.float32)
    return out


def discounted_returns(rewards, dones, gamma):
    """[T] rewards/dones of one env stream -> discounted return-to-go, reset at dones."""
    out = np.zeros(len(rewards), np.float32)
    run = 0.0
    for t in range(len(rewards) - 1, -1, -1):
        if dones[t]:
            run = 0.0
        run = rewards[t] + gamma * run
        out[t] = run
    return out


def _fragment_file_block(fn: str, file_index: int) -> dict:
    streams = _Streams(file_index)
    parts = [fragment_to_transitions(b, streams) for b in read_fragments(fn)]
    parts = [p for p in parts if len(p["rewards"])]
    if not parts:
        return {}
    keys = [k for k in parts[0] if all(k in p for p in parts)]
    return {k: np.concatenate([p[k] for p in parts]) for k in keys}


def read_offline_dataset(inp, *, read_method: str | None = None, read_kwargs=None):
    """Recorded experience as a ray_amd.data Dataset of transition rows.

    ``inp``: a directory, file, glob or list of them. ``read_method``: "read_parquet"
    (transition rows), "read_json" (fragment JSON lines) or None to pick by extension.
    Reading runs as Ray Data read tasks (one per file), so the rows stream through the
    object store to whichever consumer iterates them."""
    from ray_amd import data as rd
    from ray_amd.data.datasource import Datasource, ReadTask

    if read_method is None:
        pq_files = _files(inp, (".parquet",))
        read_method = "read_parquet" if pq_files else "read_json"
    if read_method == "read_parquet":
        return rd.read_parquet(inp if not isinstance(inp, (list, tuple)) else list(inp),
                               **(read_kwargs or {}))
    if read_method != "read_json":
        raise ValueError(f"unsupported offline read_method {read_method!r}")
    files = _files(inp)
    if not files:
        raise FileNotFoundError(f"no offline data files under {inp!r}")

    class FragmentJsonDatasource(Datasource):
        def get_read_tasks(self, parallelism):
            return [ReadTask(lambda f=f, i=i: _fragment_file_block(f, i + 1),
                             {"input_files": [f]}) for i, f in enumerate(files)]

    return rd.read_datasource(FragmentJsonDatasource())
