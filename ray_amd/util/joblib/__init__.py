"""joblib on ray_amd: ``register_ray()`` then ``with joblib.parallel_backend("ray"): ...``.

Reference parity: python/ray/util/joblib/__init__.py (register_ray) and ray_backend.py.
The reference re-parents joblib's multiprocessing backend onto ``ray.util.multiprocessing
.Pool``; here the backend is a native joblib ``submit``/future backend: every joblib
batch (a picklable ``BatchedCalls``) becomes one ray_amd task, whose ObjectRef future
carries joblib's completion callback — no pool actors, no polling thread, and joblib's
auto-batching sizes the tasks from measured batch durations.
"""

from __future__ import annotations


def register_ray():
    """Register the ray_amd backend under the name "ray" (joblib.parallel_backend("ray"))."""
    from joblib.parallel import register_parallel_backend

    from .ray_backend import RayBackend

    register_parallel_backend("ray", RayBackend)


__all__ = ["register_ray"]
