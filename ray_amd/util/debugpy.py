"""``ray.util.debugpy`` (reference: python/ray/util/debugpy.py): attach the debugpy (VS
Code) debugger to a worker — implemented in ``util/ray_debugpy.py``."""

from ray_amd.util.ray_debugpy import (_is_ray_debugger_post_mortem_enabled,  # noqa: F401
                                      _post_mortem, set_trace)
