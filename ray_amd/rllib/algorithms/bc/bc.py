"""``BC`` / ``BCConfig`` (reference: python/ray/rllib/algorithms/bc/bc.py): MARWIL with
beta = 0 (algorithms/marwil/marwil.py)."""

from ray_amd.rllib.algorithms.marwil.marwil import BC, BCConfig  # noqa: F401
