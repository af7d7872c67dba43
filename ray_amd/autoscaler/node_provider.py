"""Node providers (reference: python/ray/autoscaler/node_provider.py interface and
_private/fake_multi_node/node_provider.py).

A provider creates / terminates nodes and tags them; the autoscaler never touches
processes or machines directly."""

from __future__ import annotations

import itertools
import threading

TAG_NODE_KIND = "ray-node-kind"        # "worker" | "head"
TAG_USER_NODE_TYPE = "ray-user-node-type"
TAG_NODE_STATUS = "ray-node-status"    # "up-to-date" | "terminated"


class NodeProvider:
    """Interface a cluster backend implements."""

    def non_terminated_nodes(self, tag_filters: dict) -> list:
        raise NotImplementedError

    def create_node(self, node_config: dict, tags: dict, count: int) -> list:
        raise NotImplementedError

    def terminate_node(self, node_id: str) -> None:
        raise NotImplementedError

    def node_tags(self, node_id: str) -> dict:
        raise NotImplementedError

    def is_running(self, node_id: str) -> bool:
        return node_id in self.non_terminated_nodes({})

    def ray_node_id(self, node_id: str) -> str | None:
        """The ray_amd node id (raylet NodeID hex) backing provider node `node_id`."""
        return None

    def terminate_nodes(self, node_ids) -> None:
        for n in node_ids:
            self.terminate_node(n)


class FakeMultiNodeProvider(NodeProvider):
    """Nodes are node agents on this machine joined to an existing head (the same
    processes ``cluster_utils.Cluster.add_node`` starts)."""

    def __init__(self, cluster):
        self.cluster = cluster  # a cluster_utils.Cluster owning the head
        self.lock = threading.Lock()
        self.nodes: dict = {}  # provider id -> (Node, tags)
        self._ids = itertools.count(1)

    def non_terminated_nodes(self, tag_filters: dict) -> list:
        with self.lock:
            return [nid for nid, (node, tags) in self.nodes.items()
                    if node.alive() and all(tags.get(k) == v for k, v in tag_filters.items())]

    def create_node(self, node_config: dict, tags: dict, count: int) -> list:
        res = dict(node_config.get("resources", {}))
        out = []
        for _ in range(count):
            node = self.cluster.add_node(
                wait=False, num_cpus=int(res.pop("CPU", 0)) if "CPU" in res else
                node_config.get("num_cpus", 1),
                num_gpus=int(res.get("GPU", 0)),
                resources={k: v for k, v in res.items() if k not in ("CPU", "GPU")},
                labels=node_config.get("labels"),
                object_store_memory=node_config.get("object_store_memory", 128 << 20))
            res = dict(node_config.get("resources", {}))
            nid = f"fake-{next(self._ids)}"
            with self.lock:
                self.nodes[nid] = (node, dict(tags, **{TAG_NODE_STATUS: "up-to-date"}))
            out.append(nid)
        return out

    def terminate_node(self, node_id: str) -> None:
        with self.lock:
            ent = self.nodes.pop(node_id, None)
        if ent is not None:
            self.cluster.remove_node(ent[0])

    def node_tags(self, node_id: str) -> dict:
        with self.lock:
            ent = self.nodes.get(node_id)
            return dict(ent[1]) if ent else {}

    def ray_node_id(self, node_id: str):
        with self.lock:
            ent = self.nodes.get(node_id)
            return ent[0].node_id if ent else None
