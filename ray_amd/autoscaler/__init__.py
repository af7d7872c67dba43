"""Autoscaler: grow and shrink a ray_amd cluster from its resource demand.

Reference: python/ray/autoscaler (StandardAutoscaler, NodeProvider,
_private/fake_multi_node/node_provider.py, sdk.request_resources). The cloud providers
are out of scope for fixed MI355X nodes; the local ``FakeMultiNodeProvider``
starts real node agents on this machine, which is what the reference uses to test the
autoscaler, and a ``NodeProvider`` subclass is the extension point for a real fleet.
"""

from ray_amd.autoscaler.autoscaler import AutoscalerConfig, NodeTypeConfig, StandardAutoscaler
from ray_amd.autoscaler.node_provider import FakeMultiNodeProvider, NodeProvider
from ray_amd.autoscaler.sdk import request_resources

__all__ = ["AutoscalerConfig", "NodeTypeConfig", "StandardAutoscaler", "NodeProvider",
           "FakeMultiNodeProvider", "request_resources"]
