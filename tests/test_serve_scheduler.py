"""Serve deployment scheduler on a two-node cluster: replicas spread over nodes and
max_replicas_per_node (modelled on python/ray/serve/tests/test_deployment_scheduler.py,
test_max_replicas_per_node.py)."""

import ray_amd as ray
from ray_amd import serve


def test_deployment_scheduler_spreads_replicas():
    from ray_amd.cluster_utils import Cluster

    c = Cluster(initialize_head=True, head_node_args={"num_cpus": 2})
    c.add_node(num_cpus=2)
    ray.init(address=c.address)
    try:
        @serve.deployment(num_replicas=2, max_replicas_per_node=1,
                          ray_actor_options={"num_cpus": 0.5})
        class Where:
            def __call__(self):
                return ray.get_runtime_context().get_node_id()

        h = serve.run(Where.bind(), name="spread", route_prefix=None)
        nodes = {h.remote().result() for _ in range(30)}
        assert len(nodes) == 2
    finally:
        serve.shutdown()
        ray.shutdown()
        c.shutdown()
