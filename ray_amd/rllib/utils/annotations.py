"""``ray.rllib.utils.annotations`` (reference path): API-stability markers and
``override``."""

from ray_amd.rllib.utils import override  # noqa: F401
from ray_amd.util.annotations import Deprecated, DeveloperAPI, PublicAPI  # noqa: F401


def OldAPIStack(obj):  # noqa: N802 - reference name
    return obj


def OverrideToImplementCustomLogic(obj):  # noqa: N802
    return obj


def OverrideToImplementCustomLogic_CallToSuperRecommended(obj):  # noqa: N802
    return obj


def ExperimentalAPI(obj):  # noqa: N802
    return obj


def is_overridden(obj) -> bool:
    """True when the bound method ``obj`` is not the one of the class that defines the
    attribute first in the MRO's base (best effort, as the reference)."""
    func = getattr(obj, "__func__", obj)
    owner = getattr(obj, "__self__", None)
    if owner is None:
        return False
    for base in type(owner).__mro__[1:]:
        f = base.__dict__.get(func.__name__)
        if f is not None:
            return f is not func
    return False
