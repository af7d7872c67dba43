"""``ray.serve.multiplex`` module path (reference: python/ray/serve/multiplex.py):
model multiplexing — ``@serve.multiplexed`` loads models per replica into an LRU of
``max_num_models_per_replica``, and ``get_multiplexed_model_id`` reads the request's model
id (the ``serve_multiplexed_model_id`` header / handle option). Implemented in
serve/api.py; routing to replicas that hold the model is in serve/handle.py."""

from ray_amd.serve.api import get_multiplexed_model_id, multiplexed  # noqa: F401

__all__ = ["multiplexed", "get_multiplexed_model_id"]
