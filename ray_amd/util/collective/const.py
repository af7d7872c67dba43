"""``ray.util.collective.const`` (reference: python/ray/util/collective/const.py)."""

# prefix of the KV keys through which a group's rank 0 publishes its rendezvous address
# (collective.py: "collective:<group>:addr" in the "collective" namespace)
NAMED_ACTOR_STORE_SUFFIX = "_unique_id_actor"
KV_NAMESPACE = "collective"


def get_store_name(group_name: str) -> str:
    """The KV key of a group's rendezvous address."""
    if not group_name:
        raise ValueError("group_name is None.")
    return f"collective:{group_name}:addr"
