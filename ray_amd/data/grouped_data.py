"""``ray.data.grouped_data`` (reference: python/ray/data/grouped_data.py): the result of
``Dataset.groupby`` (aggregate / count / sum / min / max / mean / std / map_groups)."""

from ray_amd.data.dataset import GroupedData  # noqa: F401

GroupedDataset = GroupedData  # the reference's older name

__all__ = ["GroupedData"]
