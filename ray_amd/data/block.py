"""Blocks (reference: python/ray/data/block.py, _internal/{arrow,pandas,table}_block.py).

Canonical block = ``dict[str, np.ndarray]`` (columnar, equal length). Columnar
numpy is what the shared-memory object store moves zero-copy (pickle-5
out-of-band buffers) and what tensor columns need (images, token ids), so it is
also the cheapest form to hand to a HIP preprocessing kernel or a pinned H2D copy.
Arrow / pandas views are produced on demand (``to_batch``).

A column may also be a ``torch.Tensor`` on a GPU (a *device block*, e.g. the output of
a HIP preprocessing UDF): returned from a task it lands in the node's HBM object store
and readers on the same node map it zero-copy (hipIpc), so GPU-preprocessed batches
reach the trainer without a host round trip."""

from __future__ import annotations

import numpy as np

Block = dict


def num_rows(b: Block) -> int:
    for v in b.values():
        return len(v)
    return 0


def _is_tensor(v):
    return type(v).__name__ in ("Tensor", "Parameter") and type(v).__module__.startswith("torch")


def _col(values):
    if isinstance(values, np.ndarray) or _is_tensor(values):
        return values
    try:
        arr = np.asarray(values)
        if arr.dtype == object and len(values) and isinstance(values[0], np.ndarray):
            try:
                return np.stack(values)
            except ValueError:
                return arr
        return arr
    except (ValueError, TypeError):
        out = np.empty(len(values), dtype=object)
        for i, v in enumerate(values):
            out[i] = v
        return out


def from_rows(rows: list) -> Block:
    if not rows:
        return {}
    if not isinstance(rows[0], dict):
        rows = [{"item": r} for r in rows]
    keys = list(rows[0].keys())
    return {k: _col([r[k] for r in rows]) for k in keys}


def to_rows(b: Block):
    keys = list(b.keys())
    n = num_rows(b)
    cols = [b[k] for k in keys]
    for i in range(n):
        yield {k: _py(c[i]) for k, c in zip(keys, cols)}


def _py(v):
    if isinstance(v, np.generic):
        return v.item()
    return v


def slice_block(b: Block, start: int, end: int) -> Block:
    return {k: v[start:end] for k, v in b.items()}


def take_idx(b: Block, idx) -> Block:
    return {k: v[idx] for k, v in b.items()}


def concat(blocks: list) -> Block:
    blocks = [b for b in blocks if b and num_rows(b) > 0]
    if not blocks:
        return {}
    if len(blocks) == 1:
        return blocks[0]
    keys = list(blocks[0].keys())
    out = {}
    for k in keys:
        parts = [b[k] for b in blocks]
        if any(_is_tensor(p) for p in parts):
            import torch

            dev = next(p.device for p in parts if _is_tensor(p))
            out[k] = torch.cat([p if _is_tensor(p) else torch.from_numpy(np.asarray(p)).to(dev)
                                for p in parts])
            continue
        try:
            out[k] = np.concatenate(parts)
        except ValueError:
            o = np.empty(sum(len(p) for p in parts), dtype=object)
            i = 0
            for p in parts:
                for v in p:
                    o[i] = v
                    i += 1
            out[k] = o
    return out


def size_bytes(b: Block) -> int:
    n = 0
    for v in b.values():
        if _is_tensor(v):
            n += v.numel() * v.element_size()
        else:
            n += v.nbytes if v.dtype != object else 64 * len(v)
    return n


def from_batch(batch) -> Block:
    """Normalise a UDF output (dict of arrays/lists, pandas, arrow) to a block."""
    if batch is None:
        return {}
    if isinstance(batch, dict):
        return {k: _col(v) for k, v in batch.items()}
    try:
        import pandas as pd

        if isinstance(batch, pd.DataFrame):
            out = {}
            for c in batch.columns:
                col = batch[c]
                v = col.to_numpy()
                if v.dtype == object and len(v) and isinstance(v[0], np.ndarray):
                    try:
                        v = np.stack(v)
                    except ValueError:
                        pass
                out[str(c)] = v
            return out
    except ImportError:
        pass
    try:
        import pyarrow as pa

        if isinstance(batch, pa.Table):
            return {c: _arrow_col_to_numpy(batch.column(c)) for c in batch.column_names}
    except ImportError:
        pass
    if isinstance(batch, list):
        return from_rows(batch)
    raise TypeError(f"cannot convert {type(batch)} to a block")


def _arrow_col_to_numpy(col):
    """Arrow column -> numpy; a (fixed-size) list column of equal-length rows becomes an
    N-d tensor column again (the form write_parquet stores tensor columns in)."""
    import pyarrow as pa

    t = col.type
    if isinstance(t, pa.ExtensionType) and t.extension_name in (
            "ray.data.arrow_tensor", "ray.data.arrow_variable_shaped_tensor"):
        # tensor extension columns (written by Ray or data/extensions): N-d numpy back
        from ray_amd.data.extensions import tensor_extension  # noqa: F401 - registers types

        chunks = col.chunks if isinstance(col, pa.ChunkedArray) else [col]
        parts = [c.to_numpy() for c in chunks]
        return np.concatenate(parts) if parts else np.empty(0)
    if (pa.types.is_list(t) or pa.types.is_large_list(t) or pa.types.is_fixed_size_list(t)) \
            and col.null_count == 0:
        try:
            c = col.combine_chunks() if hasattr(col, "combine_chunks") else col
            flat = c.flatten()
            n = len(c)
            if n and len(flat) % n == 0:
                offs = np.asarray(c.offsets) if hasattr(c, "offsets") else None
                if offs is None or np.all(np.diff(offs) == len(flat) // n):
                    inner = _arrow_col_to_numpy(flat)
                    if inner.dtype != object:
                        return inner.reshape((n, len(flat) // n) + inner.shape[1:])
        except Exception:  # noqa: BLE001 - fall back to per-row conversion
            pass
    try:
        return _col(col.to_numpy(zero_copy_only=False)) if hasattr(col, "to_numpy") \
            else _col(col.to_pylist())
    except Exception:
        v = col.to_pylist()
        return _col(v)


def _np_to_arrow(v):
    """numpy column -> arrow: an N-d numeric tensor column becomes nested fixed-size lists
    (read back as the same tensor by _arrow_col_to_numpy)."""
    import pyarrow as pa

    if _is_tensor(v):
        v = v.detach().cpu().numpy()
    v = np.asarray(v)
    if v.ndim <= 1 or v.dtype == object:
        return pa.array(list(v)) if v.ndim > 1 else pa.array(v)
    arr = pa.array(np.ascontiguousarray(v).reshape(-1))
    for d in reversed(v.shape[1:]):
        arr = pa.FixedSizeListArray.from_arrays(arr, int(d))
    return arr


def to_batch(b: Block, batch_format: str = "numpy"):
    if batch_format in ("numpy", "default", None):
        return b
    if batch_format == "pandas":
        import pandas as pd

        return pd.DataFrame({k: (list(v) if v.ndim > 1 else v) for k, v in b.items()})
    if batch_format == "pyarrow":
        import pyarrow as pa

        cols = {}
        for k, v in b.items():
            cols[k] = _np_to_arrow(v)
        return pa.table(cols)
    raise ValueError(f"unknown batch_format {batch_format}")


def schema_of(b: Block) -> dict:
    return {k: (v.dtype, v.shape[1:]) for k, v in b.items()}


class Schema:
    def __init__(self, s: dict):
        self._s = s
        self.names = list(s.keys())
        self.types = [str(t) + (str(list(sh)) if sh else "") for t, sh in s.values()]

    def __repr__(self):
        inner = ", ".join(f"{n}: {t}" for n, t in zip(self.names, self.types))
        return f"Column names & types: {{{inner}}}"

    def __eq__(self, o):
        return isinstance(o, Schema) and o.names == self.names and o.types == self.types
