"""Preprocessors (reference: python/ray/data/preprocessor.py, preprocessors/*).

``fit`` computes statistics with distributed aggregations; ``transform`` is a
map_batches stage. ``GPUImageNormalize`` runs the HIP uint8→normalised NCHW
kernel (ops/csrc/preprocess.hip) inside an actor pool that holds a GPU."""

from __future__ import annotations

import os
from enum import Enum

import numpy as np


class PreprocessorNotFittedException(RuntimeError):
    """``transform`` called on a fittable preprocessor that was never fitted."""


class Preprocessor:
    class FitStatus(str, Enum):
        NOT_FITTABLE = "NOT_FITTABLE"
        NOT_FITTED = "NOT_FITTED"
        PARTIALLY_FITTED = "PARTIALLY_FITTED"  # a Chain with some stages fitted
        FITTED = "FITTED"

    _is_fittable = True

    def __init__(self):
        self.stats_ = None

    def fit_status(self) -> "Preprocessor.FitStatus":
        if not self._is_fittable:
            return Preprocessor.FitStatus.NOT_FITTABLE
        return Preprocessor.FitStatus.FITTED if self.stats_ is not None else \
            Preprocessor.FitStatus.NOT_FITTED

    def fit(self, ds):
        if self._is_fittable:
            self._fit(ds)
        return self

    def fit_transform(self, ds):
        return self.fit(ds).transform(ds)

    def _check_fitted(self):
        if self.fit_status() in (Preprocessor.FitStatus.NOT_FITTED,
                                 Preprocessor.FitStatus.PARTIALLY_FITTED):
            raise PreprocessorNotFittedException(
                f"{type(self).__name__} must be fitted before transform")

    def transform(self, ds):
        self._check_fitted()
        return ds.map_batches(self._transform_numpy, batch_format="numpy", batch_size=4096)

    def transform_batch(self, batch):
        """One in-memory batch: a dict of arrays, or a pandas DataFrame (returned as one)."""
        self._check_fitted()
        try:
            import pandas as pd
        except ImportError:  # pragma: no cover
            pd = None
        if pd is not None and isinstance(batch, pd.DataFrame):
            out = self._transform_numpy({c: batch[c].to_numpy() for c in batch.columns})
            return pd.DataFrame({k: (list(v) if getattr(v, "ndim", 1) > 1 else v)
                                 for k, v in out.items()})
        return self._transform_numpy(dict(batch))

    def serialize(self) -> str:
        """This (fitted) preprocessor as a string (cloudpickle, base64)."""
        import base64

        import cloudpickle

        return base64.b64encode(cloudpickle.dumps(self)).decode()

    @staticmethod
    def deserialize(serialized: str) -> "Preprocessor":
        import base64

        import cloudpickle

        return cloudpickle.loads(base64.b64decode(serialized))

    def _fit(self, ds):
        pass

    def _transform_numpy(self, batch):
        raise NotImplementedError

    def __repr__(self):
        return f"{type(self).__name__}()"


class StandardScaler(Preprocessor):
    def __init__(self, columns):
        super().__init__()
        self.columns = list(columns)

    def _fit(self, ds):
        a = ds._aggregate(self.columns)
        self.stats_ = {c: (a[c]["mean"], a[c]["std"] if a[c]["n"] > 1 else 1.0)
                       for c in self.columns}

    def _transform_numpy(self, b):
        b = dict(b)
        for c in self.columns:
            m, s = self.stats_[c]
            b[c] = (b[c] - m) / (s if s else 1.0)
        return b


class MinMaxScaler(Preprocessor):
    def __init__(self, columns):
        super().__init__()
        self.columns = list(columns)

    def _fit(self, ds):
        a = ds._aggregate(self.columns)
        self.stats_ = {c: (a[c]["min"], a[c]["max"]) for c in self.columns}

    def _transform_numpy(self, b):
        b = dict(b)
        for c in self.columns:
            lo, hi = self.stats_[c]
            b[c] = (b[c] - lo) / ((hi - lo) or 1.0)
        return b


class MaxAbsScaler(Preprocessor):
    def __init__(self, columns):
        super().__init__()
        self.columns = list(columns)

    def _fit(self, ds):
        a = ds._aggregate(self.columns)
        self.stats_ = {c: max(abs(a[c]["min"]), abs(a[c]["max"])) for c in self.columns}

    def _transform_numpy(self, b):
        b = dict(b)
        for c in self.columns:
            b[c] = b[c] / (self.stats_[c] or 1.0)
        return b


class Normalizer(Preprocessor):
    _is_fittable = False

    def __init__(self, columns, norm="l2"):
        super().__init__()
        self.columns = list(columns)
        self.norm = norm

    def _transform_numpy(self, b):
        b = dict(b)
        x = np.stack([b[c].astype(np.float64) for c in self.columns], 1)
        n = {"l1": np.abs(x).sum(1), "l2": np.sqrt((x ** 2).sum(1)), "max": np.abs(x).max(1)
             }[self.norm]
        n[n == 0] = 1
        for i, c in enumerate(self.columns):
            b[c] = x[:, i] / n
        return b


class SimpleImputer(Preprocessor):
    def __init__(self, columns, strategy="mean", fill_value=None):
        super().__init__()
        self.columns = list(columns)
        self.strategy = strategy
        self.fill_value = fill_value
        self._is_fittable = strategy != "constant"

    def _fit(self, ds):
        vals = {c: [] for c in self.columns}
        for b in ds.iter_batches(batch_size=None):
            for c in self.columns:
                v = b[c].astype(np.float64)
                vals[c].append(v[~np.isnan(v)])
        self.stats_ = {}
        for c, vs in vals.items():
            v = np.concatenate(vs) if vs else np.array([0.0])
            if self.strategy == "mean":
                self.stats_[c] = float(v.mean())
            else:
                u, cnt = np.unique(v, return_counts=True)
                self.stats_[c] = float(u[cnt.argmax()])

    def transform(self, ds):
        if not self._is_fittable:
            self.stats_ = {c: self.fill_value for c in self.columns}
        return super().transform(ds)

    def _transform_numpy(self, b):
        b = dict(b)
        for c in self.columns:
            v = b[c].astype(np.float64).copy()
            v[np.isnan(v)] = self.stats_[c]
            b[c] = v
        return b


class OrdinalEncoder(Preprocessor):
    def __init__(self, columns):
        super().__init__()
        self.columns = list(columns)

    def _fit(self, ds):
        self.stats_ = {c: {v: i for i, v in enumerate(ds.unique(c))} for c in self.columns}

    def _transform_numpy(self, b):
        b = dict(b)
        for c in self.columns:
            m = self.stats_[c]
            b[c] = np.array([m.get(x.item() if isinstance(x, np.generic) else x, -1)
                             for x in b[c]], dtype=np.int64)
        return b


class LabelEncoder(OrdinalEncoder):
    def __init__(self, label_column):
        super().__init__([label_column])
        self.label_column = label_column

    def inverse_transform_batch(self, b):
        inv = {i: v for v, i in self.stats_[self.label_column].items()}
        b = dict(b)
        b[self.label_column] = np.array([inv[int(i)] for i in b[self.label_column]])
        return b


class OneHotEncoder(Preprocessor):
    def __init__(self, columns, max_categories=None):
        super().__init__()
        self.columns = list(columns)

    def _fit(self, ds):
        self.stats_ = {c: ds.unique(c) for c in self.columns}

    def _transform_numpy(self, b):
        b = dict(b)
        for c in self.columns:
            cats = self.stats_[c]
            idx = {v: i for i, v in enumerate(cats)}
            oh = np.zeros((len(b[c]), len(cats)), dtype=np.int8)
            for r, x in enumerate(b[c]):
                j = idx.get(x.item() if isinstance(x, np.generic) else x)
                if j is not None:
                    oh[r, j] = 1
            b[c] = oh
        return b


class Concatenator(Preprocessor):
    _is_fittable = False

    def __init__(self, columns=None, output_column_name="concat_out", dtype=np.float32,
                 exclude=None):
        super().__init__()
        self.columns = columns
        self.out = output_column_name
        self.dtype = dtype
        self.exclude = exclude or []

    def _transform_numpy(self, b):
        b = dict(b)
        cols = self.columns or [c for c in b if c not in self.exclude]
        parts = [b[c].reshape(len(b[c]), -1).astype(self.dtype) for c in cols]
        for c in cols:
            del b[c]
        b[self.out] = np.concatenate(parts, 1)
        return b


class BatchMapper(Preprocessor):
    _is_fittable = False

    def __init__(self, fn, batch_format="numpy", batch_size=4096):
        super().__init__()
        self.fn = fn
        self.batch_format = batch_format
        self.batch_size = batch_size

    def transform(self, ds):
        return ds.map_batches(self.fn, batch_format=self.batch_format, batch_size=self.batch_size)

    def _transform_numpy(self, b):
        return self.fn(b)


class Chain(Preprocessor):
    def __init__(self, *preprocessors):
        super().__init__()
        self.preprocessors = preprocessors

    def fit_status(self):
        st = [p.fit_status() for p in self.preprocessors]
        F = Preprocessor.FitStatus
        fittable = [x for x in st if x != F.NOT_FITTABLE]
        if not fittable:
            return F.NOT_FITTABLE
        if all(x == F.FITTED for x in fittable):
            return F.FITTED
        return F.NOT_FITTED if all(x == F.NOT_FITTED for x in fittable) else \
            F.PARTIALLY_FITTED

    def fit(self, ds):
        for p in self.preprocessors:
            ds = p.fit_transform(ds)
        self.stats_ = True
        return self

    def transform(self, ds):
        for p in self.preprocessors:
            ds = p.transform(ds)
        return ds

    def transform_batch(self, b):
        for p in self.preprocessors:
            b = p.transform_batch(b)
        return b


class TorchVisionPreprocessor(Preprocessor):
    """Apply a torchvision-style transform (tensor or ndarray in, tensor or ndarray out) to
    image columns, per image or (``batched=True``) to the whole (B, H, W, C) batch
    (reference: data/preprocessors/torch.py). Any callable works; torchvision itself is not
    needed (not installed here)."""

    _is_fittable = False

    def __init__(self, columns, transform, output_columns=None, batched: bool = False):
        super().__init__()
        output_columns = output_columns or columns
        if len(columns) != len(output_columns):
            raise ValueError(f"The length of columns should match the length of "
                             f"output_columns: {columns} vs {output_columns}.")
        self._columns, self._output_columns = list(columns), list(output_columns)
        self._fn, self._batched = transform, batched

    def _apply(self, arr):
        import torch

        try:
            out = self._fn(torch.as_tensor(np.ascontiguousarray(arr)))
        except TypeError:
            out = self._fn(arr)
        if isinstance(out, torch.Tensor):
            out = out.detach().cpu().numpy()
        if not isinstance(out, np.ndarray):
            raise ValueError("TorchVisionPreprocessor expected the transform to return a "
                             f"torch.Tensor or np.ndarray, got {type(out).__name__}")
        return out

    def _transform_numpy(self, b):
        b = dict(b)
        for c, oc in zip(self._columns, self._output_columns):
            col = b[c]
            if self._batched:
                b[oc] = self._apply(np.asarray(col))
            else:
                outs = [self._apply(x) for x in col]
                if outs and all(o.shape == outs[0].shape for o in outs):
                    b[oc] = np.stack(outs)
                else:
                    arr = np.empty(len(outs), dtype=object)
                    arr[:] = outs
                    b[oc] = arr
        return b

    def __repr__(self):
        return (f"TorchVisionPreprocessor(columns={self._columns}, "
                f"output_columns={self._output_columns}, transform={self._fn!r})")


class _GPUNormalizeUDF:
    def __init__(self, column, mean, std, out_dtype, resize, keep_on_device=False):
        import torch

        self.keep_on_device = keep_on_device
        self.column, self.mean, self.std = column, mean, std
        self.dtype = torch.bfloat16 if out_dtype == "bf16" else torch.float32
        self.resize = resize
        self.dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
        self.pin_store = os.environ.get("RAY_AMD_DATA_PIN_STORE", "0") == "1"

    def __call__(self, batch):
        import torch

        from ray_amd.ops import functional as rf

        src = np.ascontiguousarray(batch[self.column])
        if self.pin_store and self.dev.type == "cuda":
            from ray_amd._private.h2d import to_device_pinned

            x = to_device_pinned(src, self.dev)  # DMA from registered store pages
        else:
            x = torch.from_numpy(src).to(self.dev, non_blocking=True)
        y = rf.image_normalize(x, self.mean, self.std, self.dtype)
        if self.resize is not None:
            y = rf.resize_bilinear(y, self.resize)
        out = dict(batch)
        if self.keep_on_device:  # device block: travels through the HBM object store
            out[self.column] = y
            return out
        arr = y.float().cpu().numpy() if self.dtype == torch.float32 else \
            y.view(torch.int16).cpu().numpy()
        out[self.column] = arr
        return out


class GPUImageNormalize(Preprocessor):
    """uint8 NHWC → (x/255 - mean)/std NCHW (+ optional bilinear resize) on the GPU via the
    HIP preprocessing kernels; runs in an actor pool so each actor keeps its HIP context."""

    _is_fittable = False

    def __init__(self, column="image", mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225),
                 out_dtype="fp32", resize=None, concurrency=1, num_gpus=1, batch_size=256,
                 keep_on_device=False):
        super().__init__()
        self.args = (column, mean, std, out_dtype, resize, keep_on_device)
        self.concurrency = concurrency
        self.num_gpus = num_gpus
        self.batch_size = batch_size

    def transform(self, ds):
        return ds.map_batches(_GPUNormalizeUDF, fn_constructor_args=self.args,
                              concurrency=self.concurrency, num_gpus=self.num_gpus,
                              batch_size=self.batch_size, batch_format="numpy")


# ---------------------------------------------------------------- text / hashing / bins
# Reference parity: python/ray/data/preprocessors/{tokenizer,vectorizer,hasher,encoder,
# scaler,transformer,discretizer}.py — same output column naming; statistics computed by
# one distributed pass (per-block partial counts / column gathers reduced in the driver).
def _tokens(x):
    return str(x).split(" ")


def _stable_hash(s: str, n: int) -> int:
    import hashlib

    return int.from_bytes(hashlib.blake2b(str(s).encode(), digest_size=8).digest(), "little") % n


def _column_values(ds, c):
    parts = [np.asarray(b[c]) for b in ds.iter_batches(batch_size=None)]
    return np.concatenate(parts) if parts else np.array([])


class Tokenizer(Preprocessor):
    """Replace each string with its token list (``tokenization_fn``, default split on " ")."""

    _is_fittable = False

    def __init__(self, columns, tokenization_fn=None, output_columns=None):
        super().__init__()
        self.columns = list(columns)
        self.tokenization_fn = tokenization_fn or _tokens
        self.output_columns = list(output_columns or self.columns)

    def _transform_numpy(self, b):
        b = dict(b)
        for c, o in zip(self.columns, self.output_columns):
            col = np.empty(len(b[c]), dtype=object)
            col[:] = [list(self.tokenization_fn(x)) for x in b[c]]
            b[o] = col
        return b


class CountVectorizer(Preprocessor):
    """Per string column, one count column ``{col}_{token}`` for each of the (top
    ``max_features``) tokens seen during fit, most frequent first."""

    def __init__(self, columns, tokenization_fn=None, max_features=None):
        super().__init__()
        self.columns = list(columns)
        self.tokenization_fn = tokenization_fn or _tokens
        self.max_features = max_features

    def _fit(self, ds):
        from collections import Counter

        stats = {}
        for c in self.columns:
            cnt = Counter()
            for b in ds.iter_batches(batch_size=None):
                for x in b[c]:
                    cnt.update(self.tokenization_fn(x))
            stats[c] = [t for t, _ in cnt.most_common(self.max_features)]
        self.stats_ = stats

    def _transform_numpy(self, b):
        from collections import Counter

        out = {k: v for k, v in b.items() if k not in self.columns}
        for c in self.columns:
            counts = [Counter(self.tokenization_fn(x)) for x in b[c]]
            for t in self.stats_[c]:
                out[f"{c}_{t}"] = np.array([k[t] for k in counts], dtype=np.int64)
        return out


class HashingVectorizer(Preprocessor):
    """Token counts hashed into ``num_features`` buckets: columns ``hash_{col}_{i}``."""

    _is_fittable = False

    def __init__(self, columns, num_features: int, tokenization_fn=None):
        super().__init__()
        self.columns = list(columns)
        self.num_features = num_features
        self.tokenization_fn = tokenization_fn or _tokens

    def _transform_numpy(self, b):
        out = {k: v for k, v in b.items() if k not in self.columns}
        for c in self.columns:
            m = np.zeros((len(b[c]), self.num_features), dtype=np.int64)
            for r, x in enumerate(b[c]):
                for t in self.tokenization_fn(x):
                    m[r, _stable_hash(t, self.num_features)] += 1
            for i in range(self.num_features):
                out[f"hash_{c}_{i}"] = m[:, i]
        return out


class FeatureHasher(Preprocessor):
    """Hash the (column name, value) of each listed column into ``num_features`` count
    columns ``hash_{i}``: numeric values add their magnitude to the name's bucket."""

    _is_fittable = False

    def __init__(self, columns, num_features: int, output_column: str | None = None):
        super().__init__()
        self.columns = list(columns)
        self.num_features = num_features
        self.output_column = output_column

    def _transform_numpy(self, b):
        n = len(next(iter(b.values()))) if b else 0
        m = np.zeros((n, self.num_features), dtype=np.float64)
        for c in self.columns:
            v = np.asarray(b[c])
            if np.issubdtype(v.dtype, np.number):
                m[:, _stable_hash(c, self.num_features)] += v
            else:
                for r, x in enumerate(v):
                    m[r, _stable_hash(f"{c}={x}", self.num_features)] += 1
        out = {k: v for k, v in b.items() if k not in self.columns}
        if self.output_column:
            out[self.output_column] = m
        else:
            for i in range(self.num_features):
                out[f"hash_{i}"] = m[:, i]
        return out


class MultiHotEncoder(Preprocessor):
    """List-valued columns -> multi-hot count vectors over the categories seen in fit."""

    def __init__(self, columns, max_categories=None):
        super().__init__()
        self.columns = list(columns)
        self.max_categories = max_categories or {}

    def _fit(self, ds):
        from collections import Counter

        stats = {}
        for c in self.columns:
            cnt = Counter()
            for b in ds.iter_batches(batch_size=None):
                for x in b[c]:
                    cnt.update(list(x))
            cats = [k for k, _ in cnt.most_common(self.max_categories.get(c))]
            stats[c] = {k: i for i, k in enumerate(sorted(cats, key=str))}
        self.stats_ = stats

    def _transform_numpy(self, b):
        b = dict(b)
        for c in self.columns:
            idx = self.stats_[c]
            m = np.zeros((len(b[c]), len(idx)), dtype=np.int64)
            for r, x in enumerate(b[c]):
                for v in x:
                    j = idx.get(v.item() if isinstance(v, np.generic) else v)
                    if j is not None:
                        m[r, j] += 1
            b[c] = m
        return b


class Categorizer(Preprocessor):
    """Columns -> pandas ``CategoricalDtype`` with the categories seen in fit (or the
    given ``dtypes``). ``transform_batch`` returns the categorical pandas frame; dataset
    blocks here are numpy column dicts, so ``transform`` keeps the values (out-of-category
    values become None) and the categorical dtype is re-applied on ``to_pandas``-side
    batches by ``transform_batch``."""

    def __init__(self, columns, dtypes=None):
        super().__init__()
        self.columns = list(columns)
        self.dtypes = dict(dtypes or {})

    def _fit(self, ds):
        import pandas as pd

        self.stats_ = {c: self.dtypes.get(c) or pd.CategoricalDtype(ds.unique(c))
                       for c in self.columns}

    def transform(self, ds):
        if self.stats_ is None:
            raise RuntimeError("Categorizer must be fitted before transform")
        return ds.map_batches(self._transform_pandas, batch_format="pandas", batch_size=4096)

    def _transform_pandas(self, df):
        df = df.copy()
        for c in self.columns:
            df[c] = df[c].astype(self.stats_[c])
        return df

    def transform_batch(self, batch):
        import pandas as pd

        return self._transform_pandas(pd.DataFrame(batch))


class RobustScaler(Preprocessor):
    """(x - median) / (q_high - q_low), quantile_range default (0.25, 0.75)."""

    def __init__(self, columns, quantile_range=(0.25, 0.75)):
        super().__init__()
        self.columns = list(columns)
        self.quantile_range = quantile_range

    def _fit(self, ds):
        lo, hi = self.quantile_range
        st = {}
        for c in self.columns:
            v = _column_values(ds, c).astype(np.float64)
            q = np.quantile(v, [lo, 0.5, hi]) if len(v) else [0.0, 0.0, 1.0]
            st[c] = (float(q[1]), float(q[2] - q[0]))
        self.stats_ = st

    def _transform_numpy(self, b):
        b = dict(b)
        for c in self.columns:
            med, iqr = self.stats_[c]
            b[c] = (np.asarray(b[c], dtype=np.float64) - med) / (iqr if iqr else 1.0)
        return b


class PowerTransformer(Preprocessor):
    """Yeo-Johnson (any sign) or Box-Cox (positive) power transform with fixed ``power``."""

    _is_fittable = False

    def __init__(self, columns, power: float, method: str = "yeo-johnson"):
        super().__init__()
        if method not in ("yeo-johnson", "box-cox"):
            raise ValueError(f"method must be yeo-johnson or box-cox, got {method!r}")
        self.columns = list(columns)
        self.power = power
        self.method = method

    def _transform_numpy(self, b):
        b = dict(b)
        lam = self.power
        for c in self.columns:
            x = np.asarray(b[c], dtype=np.float64)
            if self.method == "box-cox":
                y = np.log(x) if lam == 0 else (np.power(x, lam) - 1) / lam
            else:
                y = np.empty_like(x)
                pos = x >= 0
                y[pos] = np.log1p(x[pos]) if lam == 0 else (np.power(x[pos] + 1, lam) - 1) / lam
                neg = ~pos
                y[neg] = -np.log1p(-x[neg]) if lam == 2 else \
                    -(np.power(1 - x[neg], 2 - lam) - 1) / (2 - lam)
            b[c] = y
        return b


class CustomKBinsDiscretizer(Preprocessor):
    """Bin index per value from user ``bins`` (edges, or {column: edges})."""

    _is_fittable = False

    def __init__(self, columns, bins, *, right=True, include_lowest=False, duplicates="raise",
                 dtypes=None):
        super().__init__()
        self.columns = list(columns)
        self.bins = bins if isinstance(bins, dict) else {c: bins for c in self.columns}
        self.right = right
        self.include_lowest = include_lowest
        self.stats_ = {}

    def _transform_numpy(self, b):
        b = dict(b)
        for c in self.columns:
            edges = np.asarray(self.bins[c], dtype=np.float64)
            x = np.asarray(b[c], dtype=np.float64)
            idx = np.searchsorted(edges, x, side="left" if self.right else "right") - 1
            if self.include_lowest:
                idx[x == edges[0]] = 0
            bad = (idx < 0) | (idx >= len(edges) - 1) | np.isnan(x)
            out = idx.astype(np.float64)
            out[bad] = np.nan
            b[c] = out
        return b


class UniformKBinsDiscretizer(CustomKBinsDiscretizer):
    """``bins`` equal-width bins between each column's fitted min and max."""

    _is_fittable = True

    def __init__(self, columns, bins, *, right=True, include_lowest=False, duplicates="raise",
                 dtypes=None):
        super().__init__(columns, {}, right=right, include_lowest=include_lowest)
        self.n_bins = bins
        self.stats_ = None

    def _fit(self, ds):
        a = ds._aggregate(self.columns)
        self.stats_ = {}
        for c in self.columns:
            k = self.n_bins[c] if isinstance(self.n_bins, dict) else self.n_bins
            lo, hi = float(a[c]["min"]), float(a[c]["max"])
            self.bins[c] = np.linspace(lo, hi, k + 1)
            self.stats_[c] = self.bins[c]
        self.include_lowest = True
