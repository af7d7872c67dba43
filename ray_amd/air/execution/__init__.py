"""Resource requests and managers for library controllers (reference:
python/ray/air/execution/resources/{request,fixed,placement_group}.py)."""
from ray_amd.air.execution.resources import (AcquiredResources,  # noqa: F401
                                             FixedAcquiredResources, FixedResourceManager,
                                             PlacementGroupAcquiredResources,
                                             PlacementGroupResourceManager, ResourceManager,
                                             ResourceRequest)
