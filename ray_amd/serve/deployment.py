"""``ray.serve.deployment`` module path (reference: python/ray/serve/deployment.py):
``Deployment`` / ``Application`` (defined in serve/api.py) and the conversions between a
deployment and its config-file schema (serve/schema.py ``DeploymentSchema``)."""

from __future__ import annotations

from ray_amd.serve.api import Application, Deployment
from ray_amd.serve.schema import DeploymentSchema

_SCHEMA_FIELDS = ("num_replicas", "max_ongoing_requests", "max_queued_requests",
                  "user_config", "autoscaling_config", "graceful_shutdown_timeout_s",
                  "health_check_period_s", "ray_actor_options")


def deployment_to_schema(d: Deployment, include_route_prefix: bool = True) -> DeploymentSchema:
    """The config-file form of ``d``'s options (code is not part of a schema)."""
    fields = {"name": d.name}
    for k in _SCHEMA_FIELDS:
        v = getattr(d, k, None)
        if k == "autoscaling_config" and v:
            v = {a: b for a, b in v.items() if a != "policy" or isinstance(b, str)}
        if v is not None and v != {}:
            fields[k] = v
    if d.autoscaling_config:  # the schema forbids both; autoscaling owns the count
        fields.pop("num_replicas", None)
    return DeploymentSchema(**fields)


def schema_to_deployment(s: DeploymentSchema) -> Deployment:
    """A code-less Deployment carrying ``s``'s options (bind it to code with ``.options``
    on the decorated deployment, as the config-file deploy path does)."""
    return Deployment(None, s.name, **s.overrides())


__all__ = ["Application", "Deployment", "deployment_to_schema", "schema_to_deployment"]
