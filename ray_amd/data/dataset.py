"""Dataset (reference: python/ray/data/dataset.py, grouped_data.py, iterator.py).

Lazy: transformations append stages to a Plan; consumption (iter_*, take, count,
write_*, materialize) runs the streaming executor. All-to-all operations
(repartition, random_shuffle, sort, groupby, union, zip, split) are map/reduce
task graphs over the materialised upstream blocks.
"""

from __future__ import annotations

import copy

import builtins
import collections
import itertools
import math
import os
import time

import numpy as np

import ray_amd as ray

from . import _executor as X
from . import block as B


class ActorPoolStrategy:
    def __init__(self, size: int | None = None, min_size: int | None = None,
                 max_size: int | None = None, max_tasks_in_flight_per_actor: int = 2):
        if size is not None:
            min_size = max_size = size
        self.min_size = min_size or 1
        self.max_size = max_size or self.min_size
        self.max_tasks_in_flight_per_actor = max_tasks_in_flight_per_actor


class TaskPoolStrategy:
    def __init__(self, size: int | None = None):
        self.size = size


# --------------------------------------------------------------------------- UDF adapters
def _batcher(fn, batch_size, batch_format, fn_args, fn_kwargs, zero_copy=False):
    def run(blk):
        n = B.num_rows(blk)
        if n == 0:
            return blk
        bs = n if batch_size in (None, "default") else int(batch_size)
        outs = []
        for s in range(0, n, bs):
            part = B.slice_block(blk, s, s + bs)
            if not zero_copy:
                part = {k: (np.array(v) if isinstance(v, np.ndarray) and not v.flags.writeable
                            else v) for k, v in part.items()}
            r = fn(B.to_batch(part, batch_format), *fn_args, **fn_kwargs)
            if hasattr(r, "__next__") and not isinstance(r, dict):
                for x in r:
                    outs.append(B.from_batch(x))
            else:
                outs.append(B.from_batch(r))
        return B.concat(outs)

    return run


def _row_map(fn, a=(), k=None):
    k = k or {}

    def run(blk):
        return B.from_rows([fn(r, *a, **k) for r in B.to_rows(blk)])

    return run


def _row_flat_map(fn, a=(), k=None):
    k = k or {}

    def run(blk):
        rows = []
        for r in B.to_rows(blk):
            rows.extend(fn(r, *a, **k))
        return B.from_rows(rows)

    return run


def _row_filter(fn, a=(), k=None):
    k = k or {}

    def run(blk):
        n = B.num_rows(blk)
        if n == 0:
            return blk
        keep = np.fromiter((bool(fn(r, *a, **k)) for r in B.to_rows(blk)), dtype=bool,
                           count=n)
        return B.take_idx(blk, np.nonzero(keep)[0])

    return run


def _compile_expr(expr: str):
    """A filter expression (reference: Dataset.filter(expr="...")) over column names,
    constants, comparisons, and/or/not, arithmetic and `in` lists, compiled to a vectorised
    numpy predicate over a batch. Anything else (calls, attributes, subscripts) is refused."""
    import ast
    import operator as op

    tree = ast.parse(expr, mode="eval")
    bins = {ast.Add: op.add, ast.Sub: op.sub, ast.Mult: op.mul, ast.Div: op.truediv,
            ast.Mod: op.mod, ast.FloorDiv: op.floordiv, ast.Pow: op.pow}
    cmps = {ast.Eq: op.eq, ast.NotEq: op.ne, ast.Lt: op.lt, ast.LtE: op.le, ast.Gt: op.gt,
            ast.GtE: op.ge}

    def ev(n, b):
        if isinstance(n, ast.Expression):
            return ev(n.body, b)
        if isinstance(n, ast.Name):
            if n.id not in b:
                raise KeyError(f"filter expression: unknown column {n.id!r}")
            return np.asarray(b[n.id])
        if isinstance(n, ast.Constant):
            return n.value
        if isinstance(n, (ast.List, ast.Tuple)):
            return [ev(e, b) for e in n.elts]
        if isinstance(n, ast.BoolOp):
            vals = [np.asarray(ev(v, b), dtype=bool) for v in n.values]
            out = vals[0]
            for v in vals[1:]:
                out = (out & v) if isinstance(n.op, ast.And) else (out | v)
            return out
        if isinstance(n, ast.UnaryOp):
            v = ev(n.operand, b)
            if isinstance(n.op, ast.Not):
                return ~np.asarray(v, dtype=bool)
            if isinstance(n.op, ast.USub):
                return -v
            if isinstance(n.op, ast.UAdd):
                return v
        if isinstance(n, ast.BinOp) and type(n.op) in bins:
            return bins[type(n.op)](ev(n.left, b), ev(n.right, b))
        if isinstance(n, ast.Compare):
            left = ev(n.left, b)
            out = None
            for o, rn in zip(n.ops, n.comparators):
                right = ev(rn, b)
                if isinstance(o, (ast.In, ast.NotIn)):
                    r = np.isin(left, np.asarray(right, dtype=object)
                                if any(isinstance(x, str) for x in right) else right)
                    r = ~r if isinstance(o, ast.NotIn) else r
                elif type(o) in cmps:
                    r = cmps[type(o)](left, right)
                else:
                    raise ValueError(f"filter expression: unsupported comparison {ast.dump(o)}")
                out = r if out is None else (out & r)
                left = right
            return out
        raise ValueError(f"filter expression: unsupported syntax {type(n).__name__} in {expr!r}")

    def run(blk):
        n = B.num_rows(blk)
        if n == 0:
            return blk
        keep = np.broadcast_to(np.asarray(ev(tree, B.to_batch(blk, "numpy")), dtype=bool),
                               (n,))
        return B.take_idx(blk, np.nonzero(keep)[0])

    return run


def _remote_res(num_cpus, num_gpus, ray_remote_args):
    """Stage resources + the remote args the executor passes through to its tasks/actors
    (memory, max_retries, scheduling_strategy, runtime_env, ...). Unknown keys raise."""
    from ._executor import PASS_THROUGH_REMOTE_ARGS

    res = {"num_cpus": num_cpus if num_cpus is not None else 1}
    if num_gpus:
        res["num_gpus"] = num_gpus
    for k, v in (ray_remote_args or {}).items():
        if k == "resources":
            if v:
                res["resources"] = v
        elif k in PASS_THROUGH_REMOTE_ARGS:
            res[k] = v
        elif k in ("num_cpus", "num_gpus"):
            res[k] = v
        else:
            raise ValueError(f"unsupported ray_remote_args key {k!r} for a Data operator")
    return res


def _make_callable_class(cls, batch_size, batch_format, ctor_args, ctor_kwargs, fn_args,
                         fn_kwargs, zero_copy):
    def make():
        inst = cls(*ctor_args, **ctor_kwargs)
        return _batcher(inst, batch_size, batch_format, fn_args, fn_kwargs, zero_copy)

    return make


# --------------------------------------------------------------------------- remote helpers
@ray.remote
def _agg_block(blk, cols, ops):
    out = {}
    for c in cols:
        v = blk.get(c)
        if v is None or len(v) == 0:
            out[c] = None
            continue
        v = v.astype(np.float64) if v.dtype != object else np.asarray(v, dtype=np.float64)
        out[c] = {"n": len(v), "sum": float(v.sum()), "sumsq": float((v * v).sum()),
                  "min": float(v.min()), "max": float(v.max())}
    return out


def _key_list(key):
    return list(key) if isinstance(key, (list, tuple)) else [key]


def _first_desc(descending):
    return bool(descending[0]) if isinstance(descending, (list, tuple)) else bool(descending)


def _lex_order(blk, keys, descending):
    """Stable lexicographic order over ``keys`` (per-key ``descending`` flags allowed):
    each key is replaced by its dense rank so any sortable dtype works."""
    if len(keys) == 1 and not isinstance(descending, (list, tuple)):
        order = np.argsort(blk[keys[0]], kind="stable")
        return order[::-1] if descending else order
    desc = list(descending) if isinstance(descending, (list, tuple)) else \
        [bool(descending)] * len(keys)
    ranks = []
    for k, d in zip(keys, desc):
        _, inv = np.unique(np.asarray(blk[k]), return_inverse=True)
        ranks.append(-inv if d else inv)
    return np.lexsort(ranks[::-1])


def _sort_key(v):
    """Total order over mixed values (numbers before strings before everything else)."""
    if isinstance(v, (bool, int, float, np.integer, np.floating)):
        return (0, float(v), "")
    if isinstance(v, str):
        return (1, 0.0, v)
    return (2, 0.0, repr(v))


def _stable_hash(x) -> int:
    """Process-independent hash (Python's str hash is salted per process, so map tasks in
    different workers would send equal keys to different partitions). Numbers that compare
    equal hash equal across dtypes (1 == 1.0 == True, as Python's hash): integral floats
    and bools hash as their int value."""
    if isinstance(x, (bool, np.bool_)):
        x = int(x)
    elif isinstance(x, (float, np.floating)) and float(x).is_integer():
        x = int(x)
    if isinstance(x, (int, np.integer)):
        return int(x) & 0x7FFFFFFFFFFFFFFF
    if isinstance(x, (float, np.floating)):
        x = float(x)  # np.float32(0.5) and 0.5 share one repr
    import zlib

    return zlib.crc32(repr(x).encode())


def _hash_keys(blk, keys):
    cols = [blk[k] for k in keys]

    def norm(x):
        return x.item() if isinstance(x, np.generic) else \
            (tuple(x) if isinstance(x, np.ndarray) else x)

    if len(cols) == 1:
        return [norm(x) for x in cols[0]]
    return [tuple(norm(x) for x in row) for row in zip(*cols)]


@ray.remote
def _partition_block(blk, n, mode, key, boundaries, seed, descending):
    rows = B.num_rows(blk)
    if n == 1:
        return blk
    if rows == 0:
        return tuple([blk] * n)
    if mode == "random":
        rng = np.random.default_rng(seed)
        assign = rng.integers(0, n, size=rows)
    elif mode == "hash":
        assign = np.array([_stable_hash(x) % n for x in _hash_keys(blk, _key_list(key))],
                          dtype=np.int64)
    elif mode == "range":  # by the first sort key; equal first keys share a partition
        assign = np.searchsorted(np.asarray(boundaries), blk[_key_list(key)[0]],
                                 side="right")
        if _first_desc(descending):
            assign = (n - 1) - assign
    else:  # contiguous split
        assign = np.minimum((np.arange(rows) * n) // rows, n - 1)
    return tuple(B.take_idx(blk, np.nonzero(assign == j)[0]) for j in range(n))


def _partition(ref, n, mode, key, boundaries, seed, descending):
    """Map side of a shuffle: one task, n output objects (never routed via the driver)."""
    out = _partition_block.options(num_returns=n).remote(ref, n, mode, key, boundaries, seed,
                                                         descending)
    return [out] if n == 1 else out


@ray.remote(num_returns=2)
def _reduce_parts(mode, key, descending, seed, *parts):
    blk = B.concat(list(parts))
    if mode == "random" and B.num_rows(blk):
        idx = np.random.default_rng(seed).permutation(B.num_rows(blk))
        blk = B.take_idx(blk, idx)
    elif mode == "range" and B.num_rows(blk):
        blk = B.take_idx(blk, _lex_order(blk, _key_list(key), descending))
    return blk, X._meta(blk)


@ray.remote
def _sample_keys(blk, key, k):
    v = blk.get(key)
    if v is None or len(v) == 0:
        return np.array([])
    idx = np.random.default_rng(0).choice(len(v), size=min(k, len(v)), replace=False)
    return np.asarray(v)[idx]


@ray.remote(num_returns=2)
def _slice_remote(blk, start, end):
    b = B.slice_block(blk, start, end)
    return b, X._meta(b)


@ray.remote(num_returns=2)
def _concat_remote(*blks):
    b = B.concat(list(blks))
    return b, X._meta(b)


@ray.remote
def _merge_parts(*parts):
    """Push-based shuffle merge: one reducer's parts of a round of map outputs."""
    parts = [p for p in parts if B.num_rows(p)]
    return B.concat(parts) if len(parts) > 1 else (parts[0] if parts else {})


def _merge_round(plist, n_out):
    return [_merge_parts.remote(*[pl[j] for pl in plist]) for j in range(n_out)]


@ray.remote(num_returns=2)
def _zip_aligned(a, *pieces):
    """Left block `a` joined with the right rows given as (ref, start, end) triples."""
    parts = [B.slice_block(pieces[i], pieces[i + 1], pieces[i + 2])
             for i in range(0, len(pieces), 3)]
    right = B.concat(parts) if len(parts) != 1 else parts[0]
    out = dict(a)
    for k, v in right.items():
        out[k if k not in out else f"{k}_1"] = v
    return out, X._meta(out)


@ray.remote(num_returns=2)
def _zip_remote(a, b):
    out = dict(a)
    for k, v in b.items():
        kk = k if k not in out else f"{k}_1"
        out[kk] = v
    return out, X._meta(out)


@ray.remote(num_returns=2)
def _groupby_reduce(key, aggs, map_fn, batch_format, *parts):
    blk = B.concat(list(parts))
    if B.num_rows(blk) == 0:
        return {}, X._meta({})
    kl = _key_list(key)
    if len(kl) == 1:
        uniq, inv = np.unique(blk[kl[0]], return_inverse=True)
    else:  # composite keys: dense ids over the key tuples, in sorted tuple order
        tuples = _hash_keys(blk, kl)
        order = sorted(set(tuples))
        idx = {t: i for i, t in enumerate(order)}
        inv = np.array([idx[t] for t in tuples], dtype=np.int64)
        uniq = order
    if map_fn is not None:
        outs = []
        for gi in range(len(uniq)):
            g = B.take_idx(blk, np.nonzero(inv == gi)[0])
            outs.append(B.from_batch(map_fn(B.to_batch(g, batch_format))))
        out = B.concat(outs)
        return out, X._meta(out)
    if len(kl) == 1:
        out = {kl[0]: uniq}
    else:
        out = {k: np.asarray([t[j] for t in uniq]) for j, k in enumerate(kl)}
    groups = [B.take_idx(blk, np.nonzero(inv == gi)[0]) for gi in range(len(uniq))]
    for agg in aggs:  # each group is whole in this partition: no merge step
        vals = [agg.finalize(agg.accumulate_block(agg.init(k), g))
                for k, g in zip(uniq, groups)]
        col = np.empty(len(vals), dtype=object)
        col[:] = vals
        try:
            col = np.asarray(vals) if all(np.isscalar(v) for v in vals) else col
        except (ValueError, TypeError):
            pass
        out[agg.name] = col
    return out, X._meta(out)


@ray.remote
def _write_block(blk, path, fmt, idx, kw):
    return _write_local(blk, path, fmt, idx, kw)


def _write_local(blk, path, fmt, idx, kw):
    kw = dict(kw)
    pcols = kw.pop("partition_cols", None)
    if pcols:
        # Hive layout (reference: write_parquet(partition_cols=...)): one file per
        # distinct value combination under col=value/... directories, without those columns
        n = B.num_rows(blk)
        if n == 0:
            return 0
        keys = list(zip(*[[str(v) for v in np.asarray(blk[c]).tolist()] for c in pcols]))
        groups: dict = {}
        for i, k in enumerate(keys):
            groups.setdefault(k, []).append(i)
        rest = {c: v for c, v in blk.items() if c not in pcols}
        for k, rows in groups.items():
            sub = os.path.join(path, *[f"{c}={v}" for c, v in zip(pcols, k)])
            _write_local(B.take_idx(rest, np.asarray(rows)), sub, fmt, idx, kw)
        return n
    os.makedirs(path, exist_ok=True)
    fp = kw.pop("filename_provider", None)
    for k in ("try_create_dir", "arrow_open_stream_args", "ray_remote_args", "concurrency",
              "num_rows_per_file", "min_rows_per_file"):
        kw.pop(k, None)
    if fp is not None:  # a datasource.FilenameProvider names the block's file
        name = fp.get_filename_for_block(blk, idx, 0)
        base = os.path.join(path, os.path.splitext(name)[0])
    else:
        base = os.path.join(path, f"part_{idx:06d}")
    if fmt == "parquet":
        import pyarrow.parquet as pq

        pq.write_table(B.to_batch(blk, "pyarrow"), base + ".parquet", **kw)
    elif fmt == "csv":
        B.to_batch(blk, "pandas").to_csv(base + ".csv", index=False, **kw)
    elif fmt == "json":
        B.to_batch(blk, "pandas").to_json(base + ".json", orient="records", lines=True, **kw)
    elif fmt == "numpy":
        np.save(base + ".npy", blk[kw["column"]])
    return B.num_rows(blk)


# --------------------------------------------------------------------------- Dataset
class Dataset:
    def __init__(self, plan: X.Plan):
        self._plan = plan
        self._name = None
        from . import DataContext

        self._context = copy.deepcopy(DataContext.get_current())

    # ------------------------------------------------------------- identity / lineage
    # reference: python/ray/data/dataset.py:231 copy, :4634 has_serializable_lineage,
    # :4654 serialize_lineage, :4745 deserialize_lineage, :4786 context
    @property
    def context(self):
        """The DataContext this Dataset was created under (a snapshot)."""
        return self._context

    @staticmethod
    def copy(ds: "Dataset", _deep_copy: bool = False, _as=None) -> "Dataset":
        """A new Dataset over the same plan (deep: the stage list and source copied too,
        the materialised cache dropped)."""
        cls = _as or type(ds)
        if _deep_copy:
            p = X.Plan(copy.copy(ds._plan.source), [copy.copy(st) for st in ds._plan.stages],
                       ds._plan.source_meta)
        else:
            p = X.Plan(ds._plan.source, list(ds._plan.stages), ds._plan.source_meta)
            p._cache = ds._plan._cache
        out = cls.__new__(cls)
        out.__dict__.update(ds.__dict__)
        out._plan = p
        return out

    def has_serializable_lineage(self) -> bool:
        """True when the dataset can be rebuilt from its lineage alone: it starts from read
        tasks (files / datasources that exist outside this cluster), not from object refs
        or in-process streams (from_items / from_numpy / union / zip / shuffle outputs)."""
        return self._plan.source[0] == "read"

    def serialize_lineage(self) -> bytes:
        """The read tasks and transformations (not the data, not any computed block) as
        bytes; ``Dataset.deserialize_lineage`` rebuilds the dataset, possibly on another
        cluster, and everything is recomputed from the source."""
        if not self.has_serializable_lineage():
            raise ValueError("Lineage-based serialization is only supported for datasets "
                             "created by read_*() APIs (no from_* inputs, unions, zips or "
                             "all-to-all outputs)")
        import cloudpickle

        p = self._plan
        return cloudpickle.dumps({"source": p.source, "stages": p.stages,
                                  "source_meta": p.source_meta, "name": self._name,
                                  "context": self._context,
                                  "input_files": getattr(self, "_input_files", None)})

    @staticmethod
    def deserialize_lineage(serialized_ds: bytes) -> "Dataset":
        """Rebuild a dataset from ``serialize_lineage`` bytes (trusted input: they hold
        the pickled read and transformation functions)."""
        import cloudpickle

        d = cloudpickle.loads(serialized_ds)
        ds = Dataset(X.Plan(d["source"], d["stages"], d["source_meta"]))
        ds._name = d.get("name")
        if d.get("context") is not None:
            ds._context = d["context"]
        if d.get("input_files"):
            ds._input_files = d["input_files"]
        return ds

    # ------------------------------------------------------------- transformations
    def _with(self, stage: X.Stage) -> "Dataset":
        return Dataset(self._plan.with_stage(stage))

    def map_batches(self, fn, *, batch_size="default", compute=None, batch_format="default",
                    zero_copy_batch=False, fn_args=None, fn_kwargs=None,
                    fn_constructor_args=None, fn_constructor_kwargs=None, num_cpus=None,
                    num_gpus=None, concurrency=None, **ray_remote_args) -> "Dataset":
        if batch_size == "default":
            batch_size = 1024
        res = _remote_res(num_cpus, num_gpus, ray_remote_args)
        is_class = isinstance(fn, type)
        if is_class or isinstance(compute, ActorPoolStrategy) or (concurrency is not None and
                                                                  is_class):
            pool = (1, 1)
            if isinstance(compute, ActorPoolStrategy):
                pool = (compute.min_size, compute.max_size)
            elif isinstance(concurrency, int):
                pool = (concurrency, concurrency)
            elif isinstance(concurrency, tuple):
                pool = concurrency
            if not is_class:
                f = fn
                fn = type("_FnWrapper", (), {"__call__": lambda self, b, *a, **k: f(b, *a, **k)})
            make = _make_callable_class(fn, batch_size, batch_format,
                                        fn_constructor_args or (), fn_constructor_kwargs or {},
                                        fn_args or (), fn_kwargs or {}, zero_copy_batch)
            return self._with(X.Stage("actor", make_fn=make, resources=res, pool=pool,
                                      name=getattr(fn, "__name__", "MapBatches")))
        return self._with(X.Stage("task", [_batcher(fn, batch_size, batch_format, fn_args or (),
                                                    fn_kwargs or {}, zero_copy_batch)],
                                  resources=res, name="MapBatches",
                                  concurrency=concurrency if isinstance(concurrency, int)
                                  else None))

    def map(self, fn, *, compute=None, num_cpus=None, num_gpus=None, concurrency=None,
            fn_args=None, fn_kwargs=None, fn_constructor_args=None, fn_constructor_kwargs=None,
            **ray_remote_args) -> "Dataset":
        if isinstance(fn, type):
            cls = fn

            fa, fk = tuple(fn_args or ()), dict(fn_kwargs or {})

            class _RowCls:
                def __init__(self, *a, **k):
                    self.inner = cls(*a, **k)

                def __call__(self, batch):
                    return B.from_rows([self.inner(r, *fa, **fk) for r in B.to_rows(batch)])

            return self.map_batches(_RowCls, batch_size=None, compute=compute, num_cpus=num_cpus,
                                    num_gpus=num_gpus, concurrency=concurrency,
                                    zero_copy_batch=True,
                                    fn_constructor_args=fn_constructor_args,
                                    fn_constructor_kwargs=fn_constructor_kwargs,
                                    **ray_remote_args)
        return self._row_stage(_row_map(fn, fn_args or (), fn_kwargs), "Map", num_cpus,
                               num_gpus, concurrency, ray_remote_args)

    def _row_stage(self, f, name, num_cpus, num_gpus, concurrency, ray_remote_args):
        res = _remote_res(num_cpus, num_gpus, ray_remote_args)
        return self._with(X.Stage("task", [f], resources=res, name=name,
                                  concurrency=concurrency if isinstance(concurrency, int)
                                  else None))

    def flat_map(self, fn, *, num_cpus=None, num_gpus=None, concurrency=None, fn_args=None,
                 fn_kwargs=None, **ray_remote_args) -> "Dataset":
        return self._row_stage(_row_flat_map(fn, fn_args or (), fn_kwargs), "FlatMap",
                               num_cpus, num_gpus, concurrency, ray_remote_args)

    def filter(self, fn=None, *, expr=None, num_cpus=None, num_gpus=None, concurrency=None,
               fn_args=None, fn_kwargs=None, **ray_remote_args) -> "Dataset":
        """Keep rows where ``fn(row)`` is true, or where the column expression ``expr``
        (e.g. ``"id > 5 and label in ['a', 'b']"``) holds, evaluated per batch with numpy."""
        if (fn is None) == (expr is None):
            raise ValueError("filter takes exactly one of fn or expr")
        f = _compile_expr(expr) if expr is not None else \
            _row_filter(fn, fn_args or (), fn_kwargs)
        return self._row_stage(f, "Filter", num_cpus, num_gpus, concurrency, ray_remote_args)

    def add_column(self, col, fn, **kw) -> "Dataset":
        def f(batch):
            batch = dict(batch)
            batch[col] = np.asarray(fn(batch))
            return batch

        return self.map_batches(f, batch_format="numpy")

    def drop_columns(self, cols, **kw) -> "Dataset":
        cols = [cols] if isinstance(cols, str) else list(cols)
        return self.map_batches(lambda b: {k: v for k, v in b.items() if k not in cols},
                                batch_size=None, zero_copy_batch=True)

    def select_columns(self, cols, **kw) -> "Dataset":
        cols = [cols] if isinstance(cols, str) else list(cols)
        return self.map_batches(lambda b: {k: b[k] for k in cols}, batch_size=None,
                                zero_copy_batch=True)

    def rename_columns(self, names: dict, **kw) -> "Dataset":
        return self.map_batches(lambda b: {names.get(k, k): v for k, v in b.items()},
                                batch_size=None, zero_copy_batch=True)

    def random_sample(self, fraction: float, *, seed=None) -> "Dataset":
        def f(b):
            n = B.num_rows(b)
            rng = np.random.default_rng(seed)
            return B.take_idx(b, np.nonzero(rng.random(n) < fraction)[0])

        return self._with(X.Stage("task", [f], resources={"num_cpus": 1}, name="RandomSample"))

    def limit(self, limit: int) -> "Dataset":
        parent = self

        def lazy():
            refs, metas, got = [], [], 0
            for r, m in X.execute(parent._plan):
                if got >= limit:
                    break
                n = m["num_rows"]
                if got + n > limit:
                    r, m2 = _slice_remote.remote(r, 0, limit - got)
                    m = ray.get(m2)
                    n = m["num_rows"]
                refs.append(r)
                metas.append(m)
                got += n
            return refs, metas

        return Dataset(X.Plan(("lazy", lazy)))

    # ------------------------------------------------------------- all-to-all
    def _blocks(self):
        return X.materialize(self._plan)

    def _shuffle(self, n_out, mode, key=None, boundaries=None, seed=None, descending=False):
        """All-to-all exchange. The map side is streamed: each upstream block is
        partitioned as soon as it is produced. With ``DataContext.use_push_based_shuffle``
        (reference: planner/exchange/push_based_shuffle_task_scheduler.py:400) map outputs
        are pushed through merge tasks every ``merge_factor`` maps, so each reducer reads
        ceil(M / merge_factor) merged inputs instead of M small ones; the reducers' output
        blocks stream to the consumer."""
        parent = self

        def stream():
            from . import DataContext

            ctx = DataContext.get_current()
            push = bool(getattr(ctx, "use_push_based_shuffle", False))
            mf = max(2, int(getattr(ctx, "push_based_shuffle_merge_factor", 8)))
            plist, merged, i = [], [], 0
            nonlocal n_out
            upstream = X.execute(parent._plan)
            if n_out is None:
                # output blocks = upstream blocks, decided now (at execution), not when the
                # shuffle was declared: from the plan when it knows, else after the
                # upstream block refs are in (the data stays in the object store)
                hint = parent._plan.num_blocks_hint()
                if hint is None:
                    upstream = list(upstream)
                    hint = len(upstream)
                n_out = max(1, hint)
            for r, _m in upstream:
                plist.append(_partition(r, n_out, mode, key, boundaries,
                                        None if seed is None else seed + i, descending))
                i += 1
                if push and len(plist) >= mf:
                    merged.append(_merge_round(plist, n_out))
                    plist = []
            if i == 0:
                return
            if push and plist:
                merged.append(_merge_round(plist, n_out))
                plist = []
            inputs = merged if push else plist
            for j in range(n_out):
                b, m = _reduce_parts.remote(mode, key, descending,
                                            None if seed is None else seed * 7919 + j,
                                            *[pl[j] for pl in inputs])
                yield b, m

        return Dataset(X.Plan(("stream", stream)))

    def random_shuffle(self, *, seed=None, num_blocks=None, **kw) -> "Dataset":
        """Lazy: nothing upstream runs until the shuffled dataset is consumed; without
        ``num_blocks`` the output has as many blocks as the upstream (decided then)."""
        return self._shuffle(num_blocks or None, "random", seed=seed if seed is not None else
                             int(time.time_ns() % (1 << 31)))

    def repartition(self, num_blocks: int, *, shuffle: bool = False, **kw) -> "Dataset":
        if shuffle:
            return self._shuffle(num_blocks, "random", seed=0)
        parent = self

        def lazy():
            refs, metas = parent._blocks()
            total = sum(m["num_rows"] for m in metas)
            bounds = [total * i // num_blocks for i in range(num_blocks + 1)]
            starts = np.cumsum([0] + [m["num_rows"] for m in metas])
            outs, oms = [], []
            for j in range(num_blocks):
                lo, hi = bounds[j], bounds[j + 1]
                pieces = []
                for i, r in enumerate(refs):
                    s, e = starts[i], starts[i + 1]
                    a, b = max(lo, s), min(hi, e)
                    if a < b:
                        pieces.append(_slice_remote.remote(r, int(a - s), int(b - s))[0])
                bl, m = _concat_remote.remote(*pieces)
                outs.append(bl)
                oms.append(m)
            return outs, ray.get(oms)

        return Dataset(X.Plan(("lazy", lazy)))

    def sort(self, key, descending=False, **kw) -> "Dataset":
        """Sort by one key or several (lexicographic; ``descending`` a bool or one flag
        per key): range-partitioned by the first key, each partition sorted by all."""
        keys = _key_list(key)
        if isinstance(descending, (list, tuple)) and len(descending) != len(keys):
            raise ValueError("descending must be a bool or one flag per sort key")
        parent = self

        def lazy():
            refs, metas = parent._blocks()
            n = max(1, len(refs))
            samples = np.concatenate([s for s in ray.get([_sample_keys.remote(r, keys[0], 64)
                                                          for r in refs]) if len(s)] or
                                     [np.array([])])
            # boundaries are sample elements at the quantile positions (no interpolation:
            # works for strings and any other sortable key type)
            srt = np.sort(samples)
            bounds = srt[(np.linspace(0, 1, n + 1)[1:-1] * (len(srt) - 1)).astype(int)] \
                if len(samples) else []
            ds = parent._shuffle(n, "range", key=keys if len(keys) > 1 else keys[0],
                                 boundaries=list(bounds), descending=descending)
            return ds._blocks()

        return Dataset(X.Plan(("lazy", lazy)))

    def groupby(self, key) -> "GroupedData":
        return GroupedData(self, key)

    def union(self, *others) -> "Dataset":
        """Streaming union (reference: operators/union_operator.py:12): every input runs
        in its own streaming executor at once; blocks are emitted input by input, in
        order, as they are produced — nothing is materialised first."""
        dss = [self] + list(others)

        def stream():
            its = [X.execute_started(d._plan) for d in dss]  # all inputs run at once
            for it in its:
                yield from it

        return Dataset(X.Plan(("stream", stream)))

    def zip(self, other) -> "Dataset":
        """Column-wise zip (reference: operators/zip_operator.py:19). Output blocks
        follow the LEFT dataset's block boundaries: for each left block the matching row
        range of the right dataset (spanning one or more right blocks) is sliced and
        joined in one task, as both sides stream — no single-block repartition."""
        a, b = self, other

        def stream():
            it_b = X.execute(b._plan)
            right = collections.deque()  # (ref, first row, rows)
            right_end = 0
            pos = 0
            for ra, ma in X.execute(a._plan):
                n = ma["num_rows"]
                need = pos + n
                while right_end < need:
                    nxt = next(it_b, None)
                    if nxt is None:
                        raise ValueError("Cannot zip datasets of different number of rows: "
                                         f"the right side ended at row {right_end}")
                    rb, mb = nxt
                    if mb["num_rows"]:
                        right.append((rb, right_end, mb["num_rows"]))
                        right_end += mb["num_rows"]
                pieces = [(r, max(pos, s0) - s0, min(need, s0 + k) - s0)
                          for r, s0, k in right if s0 < need and s0 + k > pos]
                while right and right[0][1] + right[0][2] <= need:
                    right.popleft()
                zb, zm = _zip_aligned.remote(ra, *[x for p in pieces for x in p])
                yield zb, zm
                pos = need
            rest = right_end - pos + sum(m["num_rows"] for _, m in it_b)
            if rest:
                raise ValueError("Cannot zip datasets of different number of rows: the "
                                 f"right side has {rest} more")

        return Dataset(X.Plan(("stream", stream)))

    def unique(self, column: str) -> list:
        """Distinct values (per-block sets in tasks, unioned on the driver). A null (None /
        NaN) counts as one distinct value, listed last (reference: groupby(column).count()
        keeps the null group)."""
        from ray_amd.data.aggregate import AggregateFn, _col, _valid

        def acc(a, blk):
            v, _ = _valid(_col(blk, column), True)
            n_null = len(np.asarray(blk[column])) - len(v)
            return (a[0] | set(v.tolist()), a[1] or n_null > 0)

        fn = AggregateFn(init=lambda k: (set(), False), accumulate_block=acc,
                         merge=lambda a, b: (a[0] | b[0], a[1] or b[1]),
                         name=f"unique({column})")
        vals, has_null = self.aggregate(fn)[f"unique({column})"] or (set(), False)
        out = sorted(vals, key=_sort_key)
        return out + [None] if has_null else out

    # ------------------------------------------------------------- splitting
    def split(self, n: int, *, equal: bool = False, locality_hints=None) -> list:
        refs, metas = self._blocks()
        if equal:
            total = sum(m["num_rows"] for m in metas)
            per = total // n
            return [self._range_subset(refs, metas, i * per, (i + 1) * per) for i in range(n)]
        groups = [[] for _ in range(n)]
        for i, (r, m) in enumerate(zip(refs, metas)):
            groups[i % n].append((r, m))
        return [Dataset(X.Plan(("refs", [r for r, _ in g]), source_meta=[m for _, m in g]))
                for g in groups]

    def _range_subset(self, refs, metas, lo, hi):
        starts = np.cumsum([0] + [m["num_rows"] for m in metas])
        out_r, out_m = [], []
        for i, r in enumerate(refs):
            s, e = starts[i], starts[i + 1]
            a, b = max(lo, s), min(hi, e)
            if a < b:
                if a == s and b == e:
                    out_r.append(r)
                    out_m.append(metas[i])
                else:
                    br, bm = _slice_remote.remote(r, int(a - s), int(b - s))
                    out_r.append(br)
                    out_m.append(ray.get(bm))
        return Dataset(X.Plan(("refs", out_r), source_meta=out_m))

    def split_at_indices(self, indices) -> list:
        refs, metas = self._blocks()
        total = sum(m["num_rows"] for m in metas)
        pts = [0] + list(indices) + [total]
        return [self._range_subset(refs, metas, pts[i], pts[i + 1]) for i in range(len(pts) - 1)]

    def split_proportionately(self, proportions) -> list:
        total = self.count()
        idx, acc = [], 0
        for p in proportions:
            acc += int(total * p)
            idx.append(acc)
        return self.split_at_indices(idx)

    def train_test_split(self, test_size, *, shuffle=False, seed=None, **kw):
        ds = self.random_shuffle(seed=seed) if shuffle else self
        total = ds.count()
        n_test = int(test_size if isinstance(test_size, int) else math.ceil(total * test_size))
        a, b = ds.split_at_indices([total - n_test])
        return a, b

    def streaming_split(self, n: int, *, equal: bool = False, locality_hints=None) -> list:
        from .iterator import SplitCoordinator, StreamSplitIterator

        coord = ray.remote(SplitCoordinator).options(
            num_cpus=0, max_concurrency=n * StreamSplitIterator.PREFETCH_BLOCKS + 2).remote(
            self._plan, n, equal)
        return [StreamSplitIterator(coord, i) for i in range(n)]

    # ------------------------------------------------------------- consumption
    def iter_internal_ref_bundles(self):
        return X.execute(self._plan)

    def iterator(self):
        from .iterator import DataIterator

        return DataIterator(self)

    def iter_batches(self, *, batch_size=256, batch_format="default", drop_last=False,
                     local_shuffle_buffer_size=None, local_shuffle_seed=None,
                     prefetch_batches=1, **kw):
        from .iterator import batch_blocks

        refs = (r for r, _ in X.execute(self._plan))
        yield from batch_blocks(refs, batch_size, batch_format, drop_last,
                                local_shuffle_buffer_size, local_shuffle_seed,
                                prefetch=prefetch_batches)

    def iter_rows(self, **kw):
        for r, _ in X.execute(self._plan):
            yield from B.to_rows(ray.get(r))

    def __iter__(self):
        return self.iter_rows()

    def iter_torch_batches(self, *, batch_size=256, dtypes=None, device="auto",
                           collate_fn=None, drop_last=False, local_shuffle_buffer_size=None,
                           local_shuffle_seed=None, prefetch_batches=1, pin_memory=True, **kw):
        from .iterator import torch_batches

        yield from torch_batches(self.iter_batches(
            batch_size=batch_size, drop_last=drop_last,
            local_shuffle_buffer_size=local_shuffle_buffer_size,
            local_shuffle_seed=local_shuffle_seed, prefetch_batches=prefetch_batches),
            dtypes, device, collate_fn, pin_memory)

    def to_torch(self, **kw):
        return self.iter_torch_batches(**kw)

    def take(self, limit: int = 20) -> list:
        out = []
        for r, _ in X.execute(self.limit(limit)._plan):
            for row in B.to_rows(ray.get(r)):
                out.append(row)
                if len(out) >= limit:
                    return out
        return out

    def take_all(self, limit=None) -> list:
        out = []
        for r, _ in X.execute(self._plan):
            out.extend(B.to_rows(ray.get(r)))
            if limit is not None and len(out) > limit:
                raise ValueError(f"The dataset has more than the given limit of {limit} rows")
        return out

    def take_batch(self, batch_size: int = 20, *, batch_format="default"):
        for b in self.limit(batch_size).iter_batches(batch_size=batch_size,
                                                     batch_format=batch_format):
            return b
        return {}

    def show(self, limit: int = 20):
        for r in self.take(limit):
            print(r)

    def count(self) -> int:
        return builtins.sum(m["num_rows"] for _, m in X.execute(self._plan))

    def schema(self):
        for r, m in X.execute(self.limit(1)._plan):
            if m and m.get("schema"):
                return B.Schema(m["schema"])
        return None

    def columns(self):
        s = self.schema()
        return s.names if s else []

    def num_blocks(self) -> int:
        return len(self._blocks()[0])

    def size_bytes(self) -> int:
        return builtins.sum(m["size_bytes"] for m in self._blocks()[1])

    def input_files(self):
        return list(getattr(self, "_input_files", []))

    def materialize(self) -> "Dataset":
        refs, metas = self._blocks()
        return MaterializedDataset(X.Plan(("refs", refs), source_meta=metas))

    def stats(self) -> str:
        refs, metas = self._blocks()
        rows = builtins.sum(m["num_rows"] for m in metas)
        head = (f"Dataset: {len(refs)} blocks, {rows} rows, "
                f"{builtins.sum(m['size_bytes'] for m in metas)} bytes; stages: "
                + " -> ".join(s.name for s in self._plan.stages))
        detail = X.format_stats(self._plan.last_stats)
        return head + ("\n" + detail if detail else "")

    def _aggregate(self, cols):
        cols = [cols] if isinstance(cols, str) else list(cols)
        parts = ray.get([_agg_block.remote(r, cols, None) for r, _ in X.execute(self._plan)])
        out = {}
        for c in cols:
            ps = [p[c] for p in parts if p[c] is not None]
            n = builtins.sum(p["n"] for p in ps)
            s = builtins.sum(p["sum"] for p in ps)
            ss = builtins.sum(p["sumsq"] for p in ps)
            out[c] = {"n": n, "sum": s, "mean": s / n if n else None,
                      "min": builtins.min(p["min"] for p in ps) if ps else None,
                      "max": builtins.max(p["max"] for p in ps) if ps else None,
                      "std": math.sqrt(max(0.0, (ss - s * s / n) / (n - 1))) if n > 1 else 0.0}
        return out

    def _single(self, on, what):
        cols = [on] if isinstance(on, str) or on is None else list(on)
        if on is None:
            cols = self.columns()
        a = self._aggregate(cols)
        vals = [a[c][what] for c in cols]
        return vals[0] if len(vals) == 1 else vals

    def _agg_cols(self, on, make):
        cols = self.columns() if on is None else ([on] if isinstance(on, str) else list(on))
        aggs = [make(c) for c in cols]
        out = self.aggregate(*aggs)
        vals = [out[a.name] for a in aggs]
        return vals[0] if len(vals) == 1 else vals

    def sum(self, on=None, ignore_nulls=True, **kw):
        return self._agg_cols(on, lambda c: Sum(c, ignore_nulls))

    def min(self, on=None, ignore_nulls=True, **kw):
        return self._agg_cols(on, lambda c: Min(c, ignore_nulls))

    def max(self, on=None, ignore_nulls=True, **kw):
        return self._agg_cols(on, lambda c: Max(c, ignore_nulls))

    def mean(self, on=None, ignore_nulls=True, **kw):
        return self._agg_cols(on, lambda c: Mean(c, ignore_nulls))

    def std(self, on=None, ddof=1, ignore_nulls=True, **kw):
        return self._agg_cols(on, lambda c: Std(c, ddof, ignore_nulls))

    def aggregate(self, *aggs):
        """All aggregations in one pass over the blocks: each task accumulates every
        AggregateFn on its block; the per-block states merge on the driver."""
        from ray_amd.data.aggregate import run_many

        return run_many(self, list(aggs))

    def to_pandas(self, limit=None):
        import pandas as pd

        blocks = [ray.get(r) for r, _ in X.execute(self._plan)]
        return B.to_batch(B.concat(blocks), "pandas") if blocks else pd.DataFrame()

    def to_numpy_refs(self, *, column=None):
        return [r for r, _ in X.execute(self._plan)]

    def to_arrow_refs(self):
        return [ray.put(B.to_batch(ray.get(r), "pyarrow")) for r, _ in X.execute(self._plan)]

    def get_internal_block_refs(self):
        return self._blocks()[0]

    # ------------------------------------------------------------- writes
    def _write(self, path, fmt, **kw):
        refs = [_write_block.remote(r, path, fmt, i, kw)
                for i, (r, _) in enumerate(X.execute(self._plan))]
        ray.get(refs)

    def write_parquet(self, path, **kw):
        self._write(path, "parquet", **kw)

    def write_csv(self, path, **kw):
        self._write(path, "csv", **kw)

    def write_json(self, path, **kw):
        self._write(path, "json", **kw)

    def write_numpy(self, path, *, column, **kw):
        self._write(path, "numpy", column=column)

    def write_datasink(self, datasink, *, ray_remote_args=None, **kw):
        """Write through a custom ``Datasink`` (data/datasource.py)."""
        from ray_amd.data.datasource import write_datasink

        return write_datasink(self, datasink, ray_remote_args)

    def write_datasource(self, datasource, *, ray_remote_args=None, **write_args):
        """Legacy form of ``write_datasink`` (reference: deprecated ``Datasource.write``
        path): a Datasink is written directly; a Datasource with a ``write(blocks)``
        method receives every block."""
        from ray_amd.data.datasource import Datasink

        if isinstance(datasource, Datasink):
            return self.write_datasink(datasource, ray_remote_args=ray_remote_args)
        blocks = [b for b in self.iter_batches(batch_size=None, batch_format="pyarrow")]
        return datasource.write(blocks, **write_args)

    # external frameworks (data/integrations.py): ImportError naming the missing package
    def to_dask(self, *a, **kw):
        from ray_amd.data import integrations

        return integrations.to_dask(self, *a, **kw)

    def to_modin(self):
        from ray_amd.data import integrations

        return integrations.to_modin(self)

    def to_mars(self):
        from ray_amd.data import integrations

        return integrations.to_mars(self)

    def to_spark(self, spark):
        from ray_amd.data import integrations

        return integrations.to_spark(self, spark)

    def to_tf(self, feature_columns, label_columns, **kw):
        from ray_amd.data import integrations

        return integrations.to_tf(self, feature_columns, label_columns, **kw)

    def iter_tf_batches(self, **kw):
        from ray_amd.data import integrations

        return integrations.iter_tf_batches(self, **kw)

    def write_bigquery(self, project_id, dataset, **kw):
        from ray_amd.data import integrations

        return integrations.write_bigquery(self, project_id, dataset, **kw)

    def write_mongo(self, uri, database, collection, **kw):
        from ray_amd.data import integrations

        return integrations.write_mongo(self, uri, database, collection, **kw)

    def write_sql(self, sql: str, connection_factory, **kw):
        """INSERT every row with ``sql`` (one DB-API placeholder per column)."""
        from ray_amd.data.datasource import SQLDatasink

        return self.write_datasink(SQLDatasink(sql, connection_factory))

    def write_webdataset(self, path: str, *, encoder: bool = True, **kw):
        """One tar shard per block; row -> members ``<__key__>.<column>``."""
        from ray_amd.data.datasource import _write_tar

        ray.get([_write_tar.remote(r, path, i, encoder)
                 for i, (r, _) in enumerate(X.execute(self._plan))])

    def write_tfrecords(self, path: str, *, tf_schema=None, compression: str | None = None,
                        **kw):
        """One TFRecord file of tf.train.Example protos per block (data/tfrecords.py);
        ``compression="gzip"`` writes ``.tfrecords.gz``."""
        from ray_amd.data.tfrecords import _write_tfrecords_block

        if tf_schema is not None:
            raise NotImplementedError("tf_schema needs tensorflow_metadata (not installed)")
        comp = compression or (kw.get("arrow_open_stream_args") or {}).get("compression")
        ray.get([_write_tfrecords_block.remote(r, path, i, comp)
                 for i, (r, _) in enumerate(X.execute(self._plan))])

    def write_images(self, path: str, column: str, file_format: str = "png", **kw):
        from ray_amd.data.datasource import _write_images_block

        ray.get([_write_images_block.remote(r, path, column, file_format, i)
                 for i, (r, _) in enumerate(X.execute(self._plan))])

    def to_random_access_dataset(self, key: str, num_workers: int | None = None):
        from ray_amd.data.random_access_dataset import RandomAccessDataset

        return RandomAccessDataset(self, key, num_workers or 2)

    def randomize_block_order(self, *, seed: int | None = None) -> "Dataset":
        """Same blocks, shuffled order (no data movement)."""
        parent = self

        def lazy():
            refs, metas = parent._blocks()
            order = np.random.default_rng(seed).permutation(len(refs))
            return [refs[i] for i in order], [metas[i] for i in order]

        return Dataset(X.Plan(("lazy", lazy)))

    def to_pandas_refs(self):
        return [ray.put(B.to_batch(ray.get(r), "pandas")) for r, _ in X.execute(self._plan)]

    def __repr__(self):
        return f"Dataset(stages={[s.name for s in self._plan.stages]})"

    def __len__(self):
        raise TypeError("Use ds.count() to compute the length of a distributed Dataset.")


class MaterializedDataset(Dataset):
    pass


class GroupedData:
    def __init__(self, ds: Dataset, key):
        self._ds = ds
        self._key = key if isinstance(key, str) else list(key)

    def _run(self, aggs=None, map_fn=None, batch_format="numpy"):
        key = self._key
        ds = self._ds
        parent = ds

        def lazy():
            refs, metas = parent._blocks()
            n = max(1, len(refs))
            plist = [_partition(r, n, "hash", key, None, None, False) for r in refs]
            outs, oms = [], []
            for j in range(n):
                b, m = _groupby_reduce.remote(key, aggs, map_fn, batch_format,
                                              *[pl[j] for pl in plist])
                outs.append(b)
                oms.append(m)
            return outs, ray.get(oms)

        return Dataset(X.Plan(("lazy", lazy))).sort(key)

    def count(self):
        return self._run([Count()])

    def sum(self, on, ignore_nulls=True):
        return self._run([Sum(on, ignore_nulls)])

    def mean(self, on, ignore_nulls=True):
        return self._run([Mean(on, ignore_nulls)])

    def min(self, on, ignore_nulls=True):
        return self._run([Min(on, ignore_nulls)])

    def max(self, on, ignore_nulls=True):
        return self._run([Max(on, ignore_nulls)])

    def std(self, on, ddof=1, ignore_nulls=True):
        return self._run([Std(on, ddof, ignore_nulls)])

    def aggregate(self, *aggs):
        return self._run(list(aggs))

    def map_groups(self, fn, *, batch_format="default", **kw):
        return self._run(None, fn, "numpy" if batch_format == "default" else batch_format)


from ray_amd.data.aggregate import (AbsMax, AggregateFn, Count, Max, Mean, Min,  # noqa: E402,F401
                                    Quantile, Std, Sum, Unique)


itertools  # noqa: B018
