"""``ray.rllib.utils.deprecation`` (reference path)."""

import functools
import warnings

from ray_amd.rllib.utils import deprecation_warning  # noqa: F401

DEPRECATED_VALUE = -1


def Deprecated(old=None, *, new=None, help=None, error=False):  # noqa: N802
    """Decorator: warn (or raise with ``error``) when the decorated object is used."""
    def deco(obj):
        name = old or getattr(obj, "__name__", str(obj))
        if isinstance(obj, type):
            init = obj.__init__

            @functools.wraps(init)
            def wrapped_init(self, *a, **k):
                deprecation_warning(name, new, help=help, error=error)
                init(self, *a, **k)

            obj.__init__ = wrapped_init
            return obj

        @functools.wraps(obj)
        def wrapped(*a, **k):
            deprecation_warning(name, new, help=help, error=error)
            return obj(*a, **k)

        return wrapped

    return deco


def deprecation_warning_once(*a, **k):
    with warnings.catch_warnings():
        warnings.simplefilter("once")
        deprecation_warning(*a, **k)
