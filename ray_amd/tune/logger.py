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


class EventFileWriter:
    """TensorBoard event files without tensorboardX / TensorFlow: ``Event`` protos
    (wall_time = 1, step = 2, file_version = 3, summary = 5; Summary.value = 1 with tag = 1,
    simple_value = 2) encoded from the protobuf wire format and framed as TFRecords by the
    native core (masked CRC32C), the layout TensorBoard reads from
    ``events.out.tfevents.<time>.<host>``."""

    def __init__(self, logdir: str, filename_suffix: str = ""):
        import socket
        import time

        os.makedirs(logdir, exist_ok=True)
        self.path = os.path.join(
            logdir, f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}"
                    f"{filename_suffix}")
        self._f = open(self.path, "ab")
        self._write_event(self._event(step=0, file_version="brain.Event:2"))

    @staticmethod
    def _event(step: int, file_version: str | None = None, scalars=None) -> bytes:
        import struct
        import time

        from ray_amd.data.tfrecords import _ld, _varint

        body = b"\x09" + struct.pack("<d", time.time())  # field 1, fixed64
        body += b"\x10" + _varint(int(step))            # field 2, varint
        if file_version is not None:
            body += _ld(3, file_version.encode())
        if scalars:
            vals = b"".join(_ld(1, _ld(1, tag.encode()) + b"\x15" + struct.pack("<f", val))
                            for tag, val in scalars)
            body += _ld(5, vals)
        return body

    def _write_event(self, ev: bytes):
        from ray_amd._native import _core

        self._f.write(_core.tfrecord_encode([ev]))
        self._f.flush()

    def add_scalars(self, step: int, scalars) -> None:
        self._write_event(self._event(step=step, scalars=list(scalars)))

    def close(self):
        self._f.close()


def read_event_file(path: str) -> list:
    """[(step, {tag: value}, file_version)] of an event file (tests / tools)."""
    import struct

    from ray_amd._native import _core
    from ray_amd.data.tfrecords import _fields

    data = open(path, "rb").read()
    out = []
    for off, n in _core.tfrecord_index(data, True):
        buf = data[off:off + n]
        step, tags, ver = 0, {}, None
        for fn, wt, v in _fields(buf):
            if fn == 2:
                step = v
            elif fn == 3:
                ver = buf[v[0]:v[1]].decode()
            elif fn == 5:
                for _, _, vspan in _fields(buf, *v):
                    tag, val = None, None
                    for kfn, _, kv in _fields(buf, *vspan):
                        if kfn == 1:
                            tag = buf[kv[0]:kv[1]].decode()
                        elif kfn == 2:
                            val = struct.unpack("<f", struct.pack("<I", kv))[0]
                    tags[tag] = val
        out.append((step, tags, ver))
    return out


class TBXLoggerCallback(LoggerCallback):
    """TensorBoard scalars per trial (reference: tune/logger/tensorboardx.py): every
    numeric result entry, flattened with '/', under ``ray/tune/<key>`` at step
    ``training_iteration``; hyper-parameters as ``config/<key>`` scalars at step 0."""

    _SKIP = {"config", "trial_id", "experiment_id", "date", "timestamp", "pid", "hostname",
             "node_ip", "done", "should_checkpoint"}

    def __init__(self):
        self._writers = {}

    def log_trial_start(self, trial):
        w = self._writers.get(id(trial))
        if w is None:
            w = self._writers[id(trial)] = EventFileWriter(_trial_dir(trial))
            params = [(f"config/{k}", float(v)) for k, v in
                      flatten_dict(dict(getattr(trial, "config", {}) or {})).items()
                      if isinstance(v, (int, float)) and not isinstance(v, bool)]
            if params:
                w.add_scalars(0, params)

    def log_trial_result(self, iteration, trial, result):
        if id(trial) not in self._writers:
            self.log_trial_start(trial)
        step = result.get("training_iteration", iteration)
        flat = flatten_dict({k: v for k, v in result.items() if k not in self._SKIP})
        vals = []
        for k, v in flat.items():
            if isinstance(v, bool) or not isinstance(v, (int, float)):
                item = getattr(v, "item", None)
                if not callable(item) or getattr(v, "ndim", 1) != 0:
                    continue
                v = item()
            if isinstance(v, (int, float)) and math.isfinite(v):
                vals.append((f"ray/tune/{k}", float(v)))
        if vals:
            self._writers[id(trial)].add_scalars(int(step), vals)

    def log_trial_end(self, trial, failed=False):
        w = self._writers.pop(id(trial), None)
        if w is not None:
            w.close()


DEFAULT_LOGGERS = (JsonLoggerCallback, CSVLoggerCallback, TBXLoggerCallback)


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


# ----------------------------------------------------------------- legacy Logger API
class _LoggerTrial:
    """The minimal trial the callback loggers need (config + directory)."""

    def __init__(self, config, logdir, trial=None):
        self.config = config or {}
        self.local_path = self.path = logdir
        self.trial_id = getattr(trial, "trial_id", os.path.basename(logdir or ""))


class Logger:
    """The reference's per-trial logger (python/ray/tune/logger/logger.py ``Logger``):
    ``on_result(result)`` per reported result, ``update_config``, ``flush``, ``close``.
    New code uses the ``LoggerCallback`` classes; these wrap them."""

    _callback_cls = None

    def __init__(self, config: dict, logdir: str, trial=None):
        self.config = config
        self.logdir = logdir
        self.trial = trial
        os.makedirs(logdir, exist_ok=True)
        self._t = _LoggerTrial(config, logdir, trial)
        self._cb = self._callback_cls() if self._callback_cls else None
        self._init()

    def _init(self):
        if self._cb is not None:
            self._cb.log_trial_start(self._t)

    def on_result(self, result: dict):
        if self._cb is not None:
            self._cb.log_trial_result(result.get("training_iteration", 0), self._t, result)

    def update_config(self, config: dict):
        self.config = self._t.config = config
        if self._cb is not None:
            self._cb.log_trial_start(self._t)

    def close(self):
        if self._cb is not None:
            self._cb.log_trial_end(self._t)

    def flush(self):
        pass


class NoopLogger(Logger):
    pass


class JsonLogger(Logger):
    _callback_cls = JsonLoggerCallback


class CSVLogger(Logger):
    _callback_cls = CSVLoggerCallback


class TBXLogger(Logger):
    _callback_cls = TBXLoggerCallback


class UnifiedLogger(Logger):
    """JSON + CSV + TensorBoard (or the ``loggers`` given)."""

    def __init__(self, config, logdir, trial=None, loggers=None):
        self._loggers = [cls(config, logdir, trial) for cls in
                         (loggers or (JsonLogger, CSVLogger, TBXLogger))]
        self.config, self.logdir, self.trial = config, logdir, trial

    def on_result(self, result):
        for lg in self._loggers:
            lg.on_result(result)

    def update_config(self, config):
        for lg in self._loggers:
            lg.update_config(config)

    def close(self):
        for lg in self._loggers:
            lg.close()

    def flush(self):
        for lg in self._loggers:
            lg.flush()


class LegacyLoggerCallback(LoggerCallback):
    """Runs ``Logger`` classes as a callback: one logger of each class per trial."""

    def __init__(self, logger_classes):
        self.logger_classes = list(logger_classes)
        self._loggers = {}

    def log_trial_start(self, trial):
        if id(trial) not in self._loggers:
            d = _trial_dir(trial)
            self._loggers[id(trial)] = [c(getattr(trial, "config", {}) or {}, d, trial)
                                        for c in self.logger_classes]
        else:
            for lg in self._loggers[id(trial)]:
                lg.update_config(getattr(trial, "config", {}) or {})

    def log_trial_result(self, iteration, trial, result):
        if id(trial) not in self._loggers:
            self.log_trial_start(trial)
        for lg in self._loggers[id(trial)]:
            lg.on_result(result)

    def log_trial_end(self, trial, failed=False):
        for lg in self._loggers.pop(id(trial), []):
            lg.close()


def pretty_print(result: dict, exclude=None) -> str:
    """A result dict as indented YAML, without ``config`` / hidden keys (reference:
    tune/logger/logger.py pretty_print)."""
    import yaml

    out = {k: _jsonable(v) for k, v in result.items()
           if k != "config" and not k.startswith("_") and k not in set(exclude or ())}
    return yaml.safe_dump(out, default_flow_style=False, sort_keys=True)
