"""ray_amd.serve — model serving (reference: python/ray/serve)."""

# the ``serve.deployment`` submodule first: importing a submodule binds its name on the
# package, so it must load before the ``deployment`` decorator below takes that name
import ray_amd.serve.deployment  # noqa: E402,F401  isort: skip

from ray_amd.serve.api import (Application, Deployment, HTTPOptions, delete, deployment,  # noqa: F401
                               get_app_handle, get_deployment_handle, get_multiplexed_model_id,
                               get_replica_context, gRPCOptions, ingress, multiplexed, run, shutdown, start,
                               status, _run)
from ray_amd.serve.batching import batch  # noqa: F401
from ray_amd.serve.handle import (DeploymentHandle, DeploymentResponse,  # noqa: F401
                                  DeploymentResponseGenerator)
