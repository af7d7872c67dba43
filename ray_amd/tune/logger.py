"""Result loggers as Tune callbacks.

API contract (reference: python/ray/tune/logger/logger.py ``LoggerCallback`` with
``log_trial_start`` / ``log_trial_result`` / ``log_trial_end``; json.py
``JsonLoggerCallback`` writing ``result.json`` + ``params.json``; csv.py:75
``CSVLoggerCallback`` writing ``progress.csv``).

Design: one open file handle per trial, kept until the trial ends; nested result dicts
are flattened with '/' (``flatten_dict``) so CSV columns are stable; a CSV whose
column set grows mid-trial is rewritten once with the union header (the reference
silently drops the new keys).
"""

from __future__ import annotations

import csv
import json
import math
import os

from ray_amd.tune.callback import Callback

EXPR_PARAM_FILE = "params.json"
EXPR_RESULT_FILE = "result.json"
EXPR_PROGRESS_FILE = "progress.csv"


def flatten_dict(d: dict, prefix: str = "", sep: str = "/") -> dict:
    out = {}
    for k, v in d.items():
        key = f"{prefix}{sep}{k}" if prefix else str(k)
        if isinstance(v, dict):
            out.update(flatten_dict(v, key, sep))
        else:
            out[key] = v
    return out


def _jsonable(v):
    if isinstance(v, float) and (math.isnan(v) or math.isinf(v)):
        return str(v)
    if isinstance(v, (int, float, str, bool)) or v is None:
        return v
    if isinstance(v, (list, tuple)):
        return [_jsonable(x) for x in v]
    if isinstance(v, dict):
        return {str(k): _jsonable(x) for k, x in v.items()}
    item = getattr(v, "item", None)
    if callable(item):
        try:
            return item()
        except Exception:  # noqa: BLE001
            pass
    return str(v)


class LoggerCallback(Callback):
    """Routes trial events to log_trial_* methods."""

    def log_trial_start(self, trial):
        pass

    def log_trial_result(self, iteration: int, trial, result: dict):
        pass

    def log_trial_end(self, trial, failed: bool = False):
        pass

    def on_trial_start(self, iteration, trials, trial, **info):
        self.log_trial_start(trial)

    def on_trial_restore(self, iteration, trials, trial, **info):
        self.log_trial_start(trial)

    def on_trial_result(self, iteration, trials, trial, result, **info):
        self.log_trial_result(iteration, trial, result)

    def on_trial_complete(self, iteration, trials, trial, **info):
        self.log_trial_end(trial, failed=False)

    def on_trial_error(self, iteration, trials, trial, **info):
        self.log_trial_end(trial, failed=True)


def _trial_dir(trial) -> str:
    d = getattr(trial, "local_path", None) or getattr(trial, "path", None)
    os.makedirs(d, exist_ok=True)
    return d


class JsonLoggerCallback(LoggerCallback):
    """``result.json`` (one JSON object per result line) + ``params.json``."""

    def __init__(self):
        self._files = {}

    def log_trial_start(self, trial):
        d = _trial_dir(trial)
        with open(os.path.join(d, EXPR_PARAM_FILE), "w") as f:
            json.dump(_jsonable(getattr(trial, "config", {}) or {}), f, indent=2,
                      sort_keys=True)
        if id(trial) not in self._files:
            self._files[id(trial)] = open(os.path.join(d, EXPR_RESULT_FILE), "a")

    def log_trial_result(self, iteration, trial, result):
        if id(trial) not in self._files:
            self.log_trial_start(trial)
        f = self._files[id(trial)]
        f.write(json.dumps(_jsonable(result), sort_keys=True) + "\n")
        f.flush()

    def log_trial_end(self, trial, failed=False):
        f = self._files.pop(id(trial), None)
        if f is not None:
            f.close()


class CSVLoggerCallback(LoggerCallback):
    """``progress.csv``: one row per result, flattened keys as columns."""

    def __init__(self):
        self._state = {}  # id(trial) -> [file, writer, fieldnames, path]

    def _open(self, trial, fields):
        path = os.path.join(_trial_dir(trial), EXPR_PROGRESS_FILE)
        exists = os.path.exists(path) and os.path.getsize(path) > 0
        f = open(path, "a", newline="")
        w = csv.DictWriter(f, fieldnames=fields, extrasaction="ignore")
        if not exists:
            w.writeheader()
        self._state[id(trial)] = [f, w, list(fields), path]

    def log_trial_result(self, iteration, trial, result):
        flat = {k: v for k, v in flatten_dict(_jsonable(result)).items() if k != "config"
                and not k.startswith("config/")}
        st = self._state.get(id(trial))
        if st is None:
            self._open(trial, list(flat))
            st = self._state[id(trial)]
        elif any(k not in st[2] for k in flat):  # widen the header, keep earlier rows
            f, _, fields, path = st
            f.close()
            with open(path, newline="") as rf:
                rows = list(csv.DictReader(rf))
            fields = fields + [k for k in flat if k not in fields]
            with open(path, "w", newline="") as wf:
                w = csv.DictWriter(wf, fieldnames=fields, extrasaction="ignore")
                w.writeheader()
                w.writerows(rows)
            self._open(trial, fields)
            st = self._state[id(trial)]
        st[1].writerow(flat)
        st[0].flush()

    def log_trial_end(self, trial, failed=False):
        st = self._state.pop(id(trial), None)
        if st is not None:
            st[0].close()


class TBXLoggerCallback(LoggerCallback):
    """TensorBoard logging needs tensorboardX, which this image does not ship."""

    def __init__(self):
        raise ImportError("TBXLoggerCallback requires tensorboardX (not installed)")


DEFAULT_LOGGERS = (JsonLoggerCallback, CSVLoggerCallback)


def default_callbacks(user: list | None) -> list:
    """User callbacks plus the default JSON/CSV loggers unless the user supplied those
    types or TUNE_DISABLE_AUTO_CALLBACK_LOGGERS=1 (reference env var)."""
    cbs = list(user or [])
    if os.environ.get("TUNE_DISABLE_AUTO_CALLBACK_LOGGERS", "0") == "1":
        return cbs
    for cls in DEFAULT_LOGGERS:
        if not any(isinstance(c, cls) for c in cbs):
            cbs.append(cls())
    return cbs
