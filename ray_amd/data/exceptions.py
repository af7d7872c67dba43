"""``ray.data.exceptions`` (reference: python/ray/data/exceptions.py).

``RayDataUserCodeException`` marks a failure inside a user function (a ``map_batches`` UDF,
a filter predicate, ...) as opposed to ``SystemException`` for failures of Ray Data itself.
``omit_traceback_stdout`` wraps a driver-side API so that such an error surfaces with the
user's traceback only."""

from __future__ import annotations

import functools
import logging
from typing import Callable

from ray_amd.exceptions import RayTaskError, UserCodeException

data_exception_logger = logging.getLogger("ray_amd.data.exception")


class RayDataUserCodeException(UserCodeException):
    """An exception raised by user code run by Ray Data."""


class SystemException(Exception):
    """An exception raised by Ray Data's own machinery."""


def omit_traceback_stdout(fn: Callable) -> Callable:
    @functools.wraps(fn)
    def handle_trace(*args, **kwargs):
        try:
            return fn(*args, **kwargs)
        except Exception as e:
            cause = getattr(e, "cause", None) if isinstance(e, RayTaskError) else None
            if isinstance(cause, UserCodeException):
                data_exception_logger.debug("user code failed", exc_info=e)
                raise cause.with_traceback(None) from None
            raise

    return handle_trace
