"""Old-stack evaluation helpers (reference: rllib/evaluation/)."""

from ray_amd.rllib.evaluation.postprocessing import (Postprocessing,  # noqa: F401
                                                     compute_advantages,
                                                     compute_gae_for_sample_batch,
                                                     discount_cumsum)
