"""Preprocessors (reference: python/ray/data/preprocessor.py, preprocessors/*).

``fit`` computes statistics with distributed aggregations; ``transform`` is a
map_batches stage. ``GPUImageNormalize`` runs the HIP uint8→normalised NCHW
kernel (ops/csrc/preprocess.hip) inside an actor pool that holds a GPU."""

from __future__ import annotations

import numpy as np


class Preprocessor:
    _is_fittable = True

    def __init__(self):
        self.stats_ = None

    def fit(self, ds):
        if self._is_fittable:
            self._fit(ds)
        return self

    def fit_transform(self, ds):
        return self.fit(ds).transform(ds)

    def transform(self, ds):
        if self._is_fittable and self.stats_ is None:
            raise RuntimeError(f"{type(self).__name__} must be fitted before transform")
        return ds.map_batches(self._transform_numpy, batch_format="numpy", batch_size=4096)

    def transform_batch(self, batch):
        return self._transform_numpy(dict(batch))

    def _fit(self, ds):
        pass

    def _transform_numpy(self, batch):
        raise NotImplementedError


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


class _GPUNormalizeUDF:
    def __init__(self, column, mean, std, out_dtype, resize, keep_on_device=False):
        import torch

        self.keep_on_device = keep_on_device
        self.column, self.mean, self.std = column, mean, std
        self.dtype = torch.bfloat16 if out_dtype == "bf16" else torch.float32
        self.resize = resize
        self.dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")

    def __call__(self, batch):
        import torch

        from ray_amd.ops import functional as rf

        x = torch.from_numpy(np.ascontiguousarray(batch[self.column])).to(self.dev,
                                                                          non_blocking=True)
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
