"""``ray.serve.dag`` module path (reference: python/ray/serve/dag.py): the DAG input
node used when binding deployment graphs."""

from ray_amd.dag import InputNode  # noqa: F401

__all__ = ["InputNode"]
