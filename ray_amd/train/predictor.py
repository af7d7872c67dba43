"""Batch inference over trained models (reference: python/ray/train/predictor.py:40,
python/ray/train/_internal/dl_predictor.py).

A ``Predictor`` turns one batch into predictions: the checkpoint's preprocessor (if any)
runs ``transform_batch`` first, then the subclass's ``_predict_numpy`` or
``_predict_pandas``. The output has the input's format: a pandas DataFrame in, a
DataFrame out; a numpy array or a dict of arrays in, a dict of arrays out. A subclass
implements whichever of the two it prefers; ``predict`` converts between formats.

Predictors are used inside ``Dataset.map_batches`` through a callable class (one model
per actor), never shipped by pickling: ``__reduce__`` raises, as in the reference, so a
multi-GB model is not serialised into every task by accident.
"""

from __future__ import annotations

import numpy as np

NUMPY, PANDAS = "numpy", "pandas"


class PredictorNotSerializableException(RuntimeError):
    """Raised when a Predictor is pickled (construct it inside the worker instead)."""


def _is_df(x) -> bool:
    try:
        import pandas as pd
    except ImportError:  # pragma: no cover
        return False
    return isinstance(x, pd.DataFrame)


def _to_pandas(batch):
    import pandas as pd

    if isinstance(batch, pd.DataFrame):
        return batch
    if isinstance(batch, np.ndarray):
        if batch.ndim == 1:
            return pd.DataFrame({"__value__": batch})
        return pd.DataFrame({"__value__": list(batch)})
    cols = {}
    for k, v in batch.items():
        v = np.asarray(v)
        cols[k] = v if v.ndim <= 1 else list(v)
    return pd.DataFrame(cols)


def _to_numpy(batch):
    """DataFrame -> dict of arrays (multi-dim cells stacked back into one ndarray)."""
    if isinstance(batch, (np.ndarray, dict)):
        return batch
    out = {}
    for c in batch.columns:
        col = batch[c].to_numpy()
        if col.dtype == object and len(col) and isinstance(col[0], np.ndarray):
            col = np.stack(col)
        out[c] = col
    if list(out) == ["__value__"]:
        return out["__value__"]
    return out


class Predictor:
    def __init__(self, preprocessor=None):
        self._preprocessor = preprocessor
        self._cast_tensor_columns = False

    @classmethod
    def from_checkpoint(cls, checkpoint, **kwargs) -> "Predictor":
        raise NotImplementedError

    @classmethod
    def from_pandas_udf(cls, pandas_udf) -> "Predictor":
        """A Predictor around a ``DataFrame -> DataFrame`` function (tests, quick jobs)."""

        class PandasUDFPredictor(Predictor):
            @classmethod
            def from_checkpoint(cls, checkpoint, **kwargs):
                return PandasUDFPredictor()

            def _predict_pandas(self, df, **kwargs):
                return pandas_udf(df, **kwargs)

        return PandasUDFPredictor()

    def get_preprocessor(self):
        return self._preprocessor

    def set_preprocessor(self, preprocessor) -> None:
        self._preprocessor = preprocessor

    @classmethod
    def preferred_batch_format(cls) -> str:
        """The format the subclass implements (pandas wins when both are overridden)."""
        if cls._predict_pandas is not Predictor._predict_pandas:
            return PANDAS
        return NUMPY

    @classmethod
    def _batch_format_to_use(cls) -> str:
        has_pd = cls._predict_pandas is not Predictor._predict_pandas
        has_np = cls._predict_numpy is not Predictor._predict_numpy
        if not (has_pd or has_np):
            raise NotImplementedError(
                f"{cls.__name__} must implement _predict_pandas or _predict_numpy")
        pref = cls.preferred_batch_format()
        if pref == PANDAS and has_pd or pref == NUMPY and has_np:
            return pref
        return PANDAS if has_pd else NUMPY

    def _set_cast_tensor_columns(self):
        self._cast_tensor_columns = True

    def predict(self, data, **kwargs):
        if not hasattr(self, "_preprocessor"):
            raise NotImplementedError(
                "Subclasses of Predictor must call Predictor.__init__(preprocessor).")
        if _is_df(data):
            fmt = PANDAS
        elif isinstance(data, (np.ndarray, dict)):
            fmt = NUMPY
        else:
            raise RuntimeError(f"Invalid input data type of {type(data)}, supported types: "
                               "numpy.ndarray, dict of numpy.ndarray, pandas.DataFrame")
        if self._preprocessor is not None:
            data = self._preprocessor.transform_batch(
                data if fmt == NUMPY and isinstance(data, dict) else _to_numpy(data))
            if fmt == PANDAS:
                data = _to_pandas(data)
        use = self._batch_format_to_use()
        if fmt == PANDAS:
            if use == PANDAS:
                return self._predict_pandas(data, **kwargs)
            return _to_pandas(self._predict_numpy(_to_numpy(data), **kwargs))
        if use == NUMPY:
            return self._predict_numpy(data, **kwargs)
        return _to_numpy(self._predict_pandas(_to_pandas(data), **kwargs))

    def _predict_pandas(self, data, **kwargs):
        raise NotImplementedError

    def _predict_numpy(self, data, **kwargs):
        raise NotImplementedError

    def __reduce__(self):
        raise PredictorNotSerializableException(
            "Predictor instances are not serializable. Construct the Predictor inside the "
            "worker, e.g. in the constructor of a callable class passed to "
            "Dataset.map_batches.")


class DLPredictor(Predictor):
    """Deep-learning predictors: numpy in, framework tensors through ``call_model``,
    numpy out (a single-column dict is unwrapped to its array first, so preprocessors
    written for training are reused unchanged)."""

    def _arrays_to_tensors(self, arrays, dtype):
        raise NotImplementedError

    def _tensor_to_array(self, tensor) -> np.ndarray:
        raise NotImplementedError

    def call_model(self, inputs):
        raise NotImplementedError

    @classmethod
    def preferred_batch_format(cls) -> str:
        return NUMPY

    def _predict_numpy(self, data, dtype=None):
        if isinstance(data, dict) and len(data) == 1:
            data = next(iter(data.values()))
        out = self.call_model(self._arrays_to_tensors(data, dtype))
        if isinstance(out, dict):
            return {k: self._tensor_to_array(v) for k, v in out.items()}
        return {"predictions": self._tensor_to_array(out)}


__all__ = ["Predictor", "DLPredictor", "PredictorNotSerializableException"]
