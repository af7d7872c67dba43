"""The "local" provider (reference: python/ray/autoscaler/local/, the on-prem provider
over a fixed list of hosts): in this framework every node of a local cluster is a process on
this machine, launched by ``ray_amd.autoscaler.sdk.create_or_update_cluster`` (the
``up`` CLI); ``FakeMultiNodeProvider`` drives autoscaling of such nodes."""

from ray_amd.autoscaler.node_provider import FakeMultiNodeProvider as LocalNodeProvider  # noqa
from ray_amd.autoscaler.sdk import (bootstrap_config, create_or_update_cluster,  # noqa: F401
                                    teardown_cluster)
