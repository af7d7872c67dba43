"""``ray.util.accelerators.accelerators`` (reference: python/ray/util/accelerators/
accelerators.py): the accelerator-type constants, defined in this package's __init__."""

from ray_amd.util.accelerators import *  # noqa: F401,F403
from ray_amd.util.accelerators import __all__ as _all  # noqa: F401
