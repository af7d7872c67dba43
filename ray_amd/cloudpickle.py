"""``ray.cloudpickle`` (the reference vendors cloudpickle; this framework uses the
installed package, the serializer of its tasks and actors)."""

from cloudpickle import *  # noqa: F401,F403
from cloudpickle import dumps, loads  # noqa: F401
