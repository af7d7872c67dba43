from ray_amd.util.multiprocessing.pool import AsyncResult, Pool  # noqa: F401
from multiprocessing import TimeoutError  # noqa: F401
