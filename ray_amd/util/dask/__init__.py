"""Dask on Ray (reference: python/ray/util/dask/__init__.py): run Dask task graphs as Ray
tasks. The scheduler works on plain dict graphs, so it runs without dask installed;
``enable_dask_on_ray`` / ``ray_dask_persist`` need dask itself."""

from ray_amd.util.dask.callbacks import (ProgressBarCallback, RayDaskCallback,  # noqa: F401
                                         local_ray_callbacks, unpack_ray_callbacks)
from ray_amd.util.dask.scheduler import (disable_dask_on_ray, enable_dask_on_ray,  # noqa: F401
                                         ray_dask_get, ray_dask_get_sync)


def ray_dask_persist(*args, **kwargs):
    """``dask.persist`` with the Ray scheduler keeping results as ObjectRefs."""
    try:
        import dask
    except ImportError as e:
        raise ImportError("ray_dask_persist needs the 'dask' package") from e
    kwargs["ray_persist"] = True
    kwargs.setdefault("scheduler", ray_dask_get)
    return dask.persist(*args, **kwargs)


__all__ = ["enable_dask_on_ray", "disable_dask_on_ray", "ray_dask_get", "ray_dask_get_sync",
           "ray_dask_persist", "RayDaskCallback", "local_ray_callbacks",
           "unpack_ray_callbacks", "ProgressBarCallback"]
