"""scikit-learn integration (reference: python/ray/train/sklearn/sklearn_checkpoint.py:16,
sklearn_predictor.py:36, sklearn_trainer.py:14).

``SklearnCheckpoint`` stores a fitted estimator (and optionally the fitted preprocessor);
``SklearnPredictor`` predicts on numpy arrays or pandas DataFrames, optionally on a
subset of ``feature_columns`` and with the estimator's thread parameters (``n_jobs``,
``thread_count``, also in nested estimators) set to ``num_estimator_cpus``, so each Data
actor uses exactly the CPUs it reserved. ``SklearnTrainer`` is deprecated upstream and
raises with the same migration advice (fit inside a Tune trainable instead).
"""

from __future__ import annotations

import os
import tempfile

import numpy as np

from ray_amd.train._checkpoint import Checkpoint
from ray_amd.train.predictor import Predictor, _is_df

SKLEARN_CPU_PARAM_NAMES = ("n_jobs", "thread_count")


class SklearnCheckpoint(Checkpoint):
    MODEL_FILENAME = "model.pkl"

    @classmethod
    def from_estimator(cls, estimator, *, path: str | None = None, preprocessor=None):
        import cloudpickle

        d = path or tempfile.mkdtemp(prefix="ra_sklearn_ckpt_")
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, cls.MODEL_FILENAME), "wb") as f:
            cloudpickle.dump(estimator, f)
        c = cls(d)
        if preprocessor is not None:
            c.set_preprocessor(preprocessor)
        return c

    def get_estimator(self):
        import pickle

        with open(os.path.join(self._local_path(), self.MODEL_FILENAME), "rb") as f:
            return pickle.load(f)


def _set_cpu_params(estimator, num_cpus: int) -> None:
    params = estimator.get_params(deep=True)
    upd = {k: num_cpus for k in params
           if k.rsplit("__", 1)[-1] in SKLEARN_CPU_PARAM_NAMES}
    if upd:
        estimator.set_params(**upd)


class SklearnPredictor(Predictor):
    def __init__(self, estimator, preprocessor=None):
        self.estimator = estimator
        super().__init__(preprocessor)

    def __repr__(self):
        return (f"{type(self).__name__}(estimator={self.estimator!r}, "
                f"preprocessor={self._preprocessor!r})")

    @classmethod
    def from_checkpoint(cls, checkpoint: SklearnCheckpoint, **kwargs) -> "SklearnPredictor":
        return cls(estimator=checkpoint.get_estimator(),
                   preprocessor=checkpoint.get_preprocessor())

    def predict(self, data, feature_columns=None, num_estimator_cpus=None, **predict_kwargs):
        """``data``: a 2-D numpy array (``feature_columns`` are column indices), a dict of
        1-D arrays or a DataFrame (``feature_columns`` are names). Returns predictions
        in the input's format: a DataFrame with a ``predictions`` column, or a dict
        ``{"predictions": array}``."""
        if self._preprocessor is not None:
            data = self._preprocessor.transform_batch(data)
        if num_estimator_cpus:
            _set_cpu_params(self.estimator, num_estimator_cpus)
        if _is_df(data):
            return self._predict_pandas(data, feature_columns=feature_columns,
                                        **predict_kwargs)
        return self._predict_numpy(data, feature_columns=feature_columns, **predict_kwargs)

    def _predict_pandas(self, df, feature_columns=None, **kw):
        import pandas as pd

        X = df[list(feature_columns)] if feature_columns else df
        y = np.asarray(self.estimator.predict(X, **kw))
        if y.ndim == 2:
            return pd.DataFrame(y, columns=[f"predictions_{i}" for i in range(y.shape[1])])
        return pd.DataFrame({"predictions": y})

    def _predict_numpy(self, data, feature_columns=None, **kw):
        if isinstance(data, dict):
            cols = list(feature_columns) if feature_columns else list(data)
            X = np.column_stack([np.asarray(data[c]) for c in cols])
        else:
            X = np.asarray(data)
            if X.ndim == 1:
                X = X[:, None]
            if feature_columns is not None:
                X = X[:, list(feature_columns)]
        return {"predictions": np.asarray(self.estimator.predict(X, **kw))}


_DEPRECATION = ("`ray_amd.train.sklearn.SklearnTrainer` is deprecated (as upstream): write "
                "your own training function and use `ray_amd.tune.Tuner` to train many "
                "sklearn models in parallel; SklearnCheckpoint / SklearnPredictor remain.")


class SklearnTrainer:
    def __new__(cls, *args, **kwargs):
        raise DeprecationWarning(_DEPRECATION)

    @classmethod
    def restore(cls, *args, **kwargs):
        raise DeprecationWarning(_DEPRECATION)

    @classmethod
    def can_restore(cls, *args, **kwargs):
        raise DeprecationWarning(_DEPRECATION)

    @staticmethod
    def get_model(*args, **kwargs):
        raise DeprecationWarning(_DEPRECATION)


__all__ = ["SklearnCheckpoint", "SklearnPredictor", "SklearnTrainer"]
