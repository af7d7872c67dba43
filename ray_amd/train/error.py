"""``ray.train.error`` (reference: python/ray/train/error.py)."""


class SessionMisuseError(RuntimeError):
    """A Train session function (``train.report``, ``train.get_context``, ...) was called
    outside a training worker. (A RuntimeError too, for callers that catch that.)"""
