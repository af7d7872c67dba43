"""Ray on Spark (reference: python/ray/util/spark/): start a Ray cluster on the executors
of a running Spark application. pyspark is not installed in this image, so the entry
points raise ImportError naming it; the cluster itself would be the ordinary ray_amd
head + node agents (``ray_amd start``) launched in Spark barrier tasks."""

MAX_NUM_WORKER_NODES = -1


def _pyspark():
    try:
        import pyspark  # noqa: F401
    except ImportError as e:
        raise ImportError("Ray on Spark needs the 'pyspark' package, which is not "
                          "installed") from e
    raise NotImplementedError("Ray on Spark: launching node agents in Spark barrier tasks "
                              "is not implemented")


def setup_ray_cluster(*args, **kwargs):
    _pyspark()


def setup_global_ray_cluster(*args, **kwargs):
    _pyspark()


def shutdown_ray_cluster():
    _pyspark()


__all__ = ["setup_ray_cluster", "setup_global_ray_cluster", "shutdown_ray_cluster",
           "MAX_NUM_WORKER_NODES"]
