"""DreamerV3 (reference: rllib/algorithms/dreamerv3)."""

from ray_amd.rllib.algorithms.dreamerv3.dreamerv3 import (MODEL_SIZES, DreamerV3,  # noqa: F401
                                                          DreamerV3Config, DreamerV3EnvRunner)

__all__ = ["DreamerV3", "DreamerV3Config", "DreamerV3EnvRunner", "MODEL_SIZES"]
