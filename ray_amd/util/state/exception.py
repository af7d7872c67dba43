"""``ray.util.state.exception`` (reference: python/ray/util/state/exception.py)."""

from ray_amd.util.state.api import RayStateApiException  # noqa: F401

DATA_SOURCE_UNAVAILABLE = "Failed to query the data source."


class DataSourceUnavailable(RayStateApiException):
    """The raylet / GCS tables the query reads could not be reached."""


class ServerUnavailable(RayStateApiException):
    """The state API server (here: the head raylet) is not running."""
