"""Tune utilities (reference: python/ray/tune/utils/util.py, exported by
tune/utils/__init__.py): nested-dict helpers, a resource monitor, save/restore and
serialization diagnostics, and ``wait_for_gpu``."""

from __future__ import annotations

import copy
import threading
import time
from datetime import datetime

import numpy as np


def date_str() -> str:
    return datetime.today().strftime("%Y-%m-%d_%H-%M-%S")


def deep_update(original: dict, new_dict: dict, new_keys_allowed: bool = False,
                allow_new_subkey_list=None, override_all_if_type_changes=None,
                override_all_key_list=None) -> dict:
    """Update ``original`` in place with ``new_dict``, recursing into dicts. Unknown keys
    raise unless ``new_keys_allowed`` (or the parent key is in ``allow_new_subkey_list``);
    a dict whose "type" changes is replaced whole when its key is in
    ``override_all_if_type_changes``."""
    allow_new_subkey_list = allow_new_subkey_list or []
    override_all_if_type_changes = override_all_if_type_changes or []
    override_all_key_list = override_all_key_list or []
    for k, v in new_dict.items():
        if k not in original and not new_keys_allowed:
            raise Exception(f"Unknown config parameter `{k}` ")
        if isinstance(original.get(k), dict) and isinstance(v, dict):
            if k in override_all_key_list or (
                    k in override_all_if_type_changes and "type" in v and
                    v["type"] != original[k].get("type")):
                original[k] = v
            else:
                deep_update(original[k], v,
                            True if k in allow_new_subkey_list else new_keys_allowed,
                            allow_new_subkey_list, override_all_if_type_changes,
                            override_all_key_list)
        else:
            original[k] = v
    return original


def merge_dicts(d1: dict, d2: dict) -> dict:
    """A deep copy of ``d1`` updated recursively with ``d2`` (new keys allowed)."""
    merged = copy.deepcopy(d1)
    deep_update(merged, d2, True, [])
    return merged


def flatten_dict(dt: dict, delimiter: str = "/", prevent_delimiter: bool = False) -> dict:
    """``{"a": {"b": 1}}`` -> ``{"a/b": 1}``."""
    out = {}

    def rec(prefix, d):
        for k, v in d.items():
            if prevent_delimiter and delimiter in str(k):
                raise ValueError(f"Found delimiter `{delimiter}` in key when trying to "
                                 f"flatten array. Please avoid using the delimiter in your "
                                 f"specification.")
            key = f"{prefix}{delimiter}{k}" if prefix else str(k)
            if isinstance(v, dict) and v:
                rec(key, v)
            else:
                out[key] = v

    rec("", dt)
    return out


def unflattened_lookup(flat_key: str, lookup, delimiter: str = "/", **kwargs):
    """``lookup["a"]["b"]`` for ``flat_key="a/b"`` (dicts and lists; ``default`` kwarg)."""
    cur = lookup
    for part in flat_key.split(delimiter):
        try:
            cur = cur[int(part)] if isinstance(cur, (list, tuple)) else cur[part]
        except (KeyError, IndexError, ValueError, TypeError):
            if "default" in kwargs:
                return kwargs["default"]
            raise
    return cur


class UtilMonitor(threading.Thread):
    """Samples CPU / RAM (psutil) and GPU utilisation (the node reporter's GPU probe)
    every ``delay`` seconds; ``get_data()`` returns the means since the last call."""

    def __init__(self, start: bool = True, delay: float = 0.7):
        super().__init__(daemon=True)
        self.delay = delay
        self.stopped = True
        self._lock = threading.Lock()
        self.values = {"cpu_util_percent": [], "ram_util_percent": [],
                       "gpu_util_percent": []}
        if start:
            self.start()

    def _sample(self):
        import psutil

        with self._lock:
            self.values["cpu_util_percent"].append(psutil.cpu_percent(interval=None))
            self.values["ram_util_percent"].append(psutil.virtual_memory().percent)
            try:
                if not hasattr(self, "_gpu"):
                    from ray_amd._private.reporter import _AmdSmi, _Sysfs

                    b = _AmdSmi()
                    self._gpu = b if b.ok else _Sysfs()
                g = [x.get("utilization_percent") for x in self._gpu.sample()]
                g = [x for x in g if x is not None]
                if g:
                    self.values["gpu_util_percent"].append(float(np.mean(g)))
            except Exception:  # noqa: BLE001 - no GPU probe on this host
                pass

    def get_data(self) -> dict:
        with self._lock:
            out = {k: float(np.mean(v)) for k, v in self.values.items() if v}
            for v in self.values.values():
                v.clear()
        return {"perf": out} if out else {}

    def run(self):
        self.stopped = False
        while not self.stopped:
            self._sample()
            time.sleep(self.delay)

    def stop(self):
        self.stopped = True


def warn_if_slow(name: str, threshold: float | None = None, disable: bool = False):
    """Context manager that prints a warning when its body takes over ``threshold`` s."""
    class _W:
        def __enter__(self):
            self.t0 = time.monotonic()
            return self

        def __exit__(self, *exc):
            dt = time.monotonic() - self.t0
            if not disable and dt > (threshold if threshold is not None else 0.5):
                print(f"The `{name}` operation took {dt:.3f} s, which may be a performance "
                      "bottleneck.")
            return False

    return _W()


def validate_save_restore(trainable_cls, config: dict | None = None,
                          num_gpus: int = 0) -> bool:
    """Checks that a class Trainable restores its state: train, save, train on a fresh
    instance restored from the checkpoint, and compare the iteration counters."""
    import tempfile

    t1 = trainable_cls(config=config or {})
    t1.train()
    with tempfile.TemporaryDirectory() as d:
        ckpt = t1.save(d)
        r1 = t1.train()
        t2 = trainable_cls(config=config or {})
        t2.restore(ckpt)
        r2 = t2.train()
    it1, it2 = r1.get("training_iteration"), r2.get("training_iteration")
    if it1 != it2:
        raise AssertionError(f"restored trainable reports iteration {it2}, expected {it1}")
    return True


def diagnose_serialization(trainable):
    """Find what in a function's closure cannot be pickled: returns True when it all
    pickles, else the set of offending names (and prints them)."""
    import inspect

    import cloudpickle

    try:
        cloudpickle.dumps(trainable)
        print("Serialization check passed.")
        return True
    except Exception as e:  # noqa: BLE001
        print(f"Trainable cannot be serialized: {e}")
    bad = set()
    if inspect.isfunction(trainable):
        cv = inspect.getclosurevars(trainable)
        for name, obj in {**cv.nonlocals, **cv.globals}.items():
            try:
                cloudpickle.dumps(obj)
            except Exception:  # noqa: BLE001
                bad.add(name)
    print(f"Variables that failed to serialize: {sorted(bad)}")
    return bad


def wait_for_gpu(gpu_id=None, target_util: float = 0.01, retry: int = 20,
                 delay_s: int = 5, gpu_memory_limit: float | None = None) -> bool:
    """Block until the (first assigned) GPU's used-memory fraction drops to
    ``target_util`` (a previous trial's process has let go of it)."""
    import torch

    if gpu_memory_limit is not None:
        target_util = gpu_memory_limit
    if not torch.cuda.is_available():
        raise RuntimeError("wait_for_gpu: no GPU is visible to this process")
    dev = int(gpu_id or 0)
    for _ in range(retry):
        free, total = torch.cuda.mem_get_info(dev)
        if (total - free) / total <= target_util:
            return True
        time.sleep(delay_s)
    raise RuntimeError(f"GPU {dev} memory did not drop to {target_util:.0%} in "
                       f"{retry * delay_s} s")


__all__ = ["deep_update", "date_str", "flatten_dict", "merge_dicts", "unflattened_lookup",
           "UtilMonitor", "validate_save_restore", "warn_if_slow", "diagnose_serialization",
           "wait_for_gpu"]
