"""ray_amd.serve — model serving (reference: python/ray/serve)."""

from ray_amd.serve.api import (Application, Deployment, HTTPOptions, delete, deployment,  # noqa: F401
                               get_app_handle, get_deployment_handle, get_multiplexed_model_id,
                               get_replica_context, gRPCOptions, ingress, multiplexed, run, shutdown, start,
                               status, _run)
from ray_amd.serve.batching import batch  # noqa: F401
from ray_amd.serve.handle import (DeploymentHandle, DeploymentResponse,  # noqa: F401
                                  DeploymentResponseGenerator)
