"""API-stability annotations: ``@PublicAPI``, ``@DeveloperAPI``, ``@Deprecated``.

Reference parity: python/ray/util/annotations.py:8,63,102. Each decorator works bare or
with arguments, records the stability level on the object (``obj._annotated``), and
prepends a note to the docstring; ``Deprecated`` also warns (``RayDeprecationWarning``)
each time a deprecated function or class is called / instantiated.
"""

from __future__ import annotations

import functools
import inspect
import warnings


class RayDeprecationWarning(DeprecationWarning):
    """Raised by APIs marked ``@Deprecated`` (shown by default, unlike DeprecationWarning)."""


warnings.simplefilter("always", RayDeprecationWarning)


def _note(obj, text: str):
    doc = obj.__doc__ or ""
    try:
        obj.__doc__ = f"{doc.rstrip()}\n\n    {text}\n" if doc else text
    except (AttributeError, TypeError):
        pass


def _mark(obj, level: str, stability: str | None = None):
    try:
        obj._annotated = obj.__qualname__ if hasattr(obj, "__qualname__") else True
        obj._annotated_type = level
        obj._annotated_stability = stability
    except (AttributeError, TypeError):
        pass
    return obj


def _decorator(make):
    """Allow ``@Deco`` and ``@Deco(...)``."""

    def deco(*args, **kwargs):
        if len(args) == 1 and not kwargs and callable(args[0]):
            return make(args[0])
        return lambda obj: make(obj, *args, **kwargs)

    return deco


@_decorator
def PublicAPI(obj, stability: str = "stable", api_group: str = "Others"):
    if stability not in ("stable", "beta", "alpha"):
        raise ValueError(f"stability must be stable, beta or alpha, not {stability!r}")
    if stability != "stable":
        _note(obj, f"PublicAPI ({stability}): This API is in {stability} and may change "
                   "before becoming stable.")
    else:
        _note(obj, "PublicAPI: This API is stable across Ray releases.")
    return _mark(obj, "PublicAPI", stability)


@_decorator
def DeveloperAPI(obj):
    _note(obj, "DeveloperAPI: This API may change across minor Ray releases.")
    return _mark(obj, "DeveloperAPI")


@_decorator
def Deprecated(obj, message: str = "", warning: bool = True):
    msg = f"DEPRECATED: This API is deprecated and may be removed in future Ray releases. " \
          f"{message}".rstrip()
    _note(obj, msg)
    if not warning:
        return _mark(obj, "Deprecated")
    if inspect.isclass(obj):
        init = obj.__init__

        @functools.wraps(init)
        def __init__(self, *a, **k):
            warnings.warn(msg, RayDeprecationWarning, stacklevel=2)
            init(self, *a, **k)

        obj.__init__ = __init__
        return _mark(obj, "Deprecated")

    @functools.wraps(obj)
    def wrapper(*a, **k):
        warnings.warn(msg, RayDeprecationWarning, stacklevel=2)
        return obj(*a, **k)

    return _mark(wrapper, "Deprecated")


def is_annotated(obj) -> bool:
    return getattr(obj, "_annotated", None) is not None
