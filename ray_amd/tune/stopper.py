"""``ray.tune.stopper`` import path (reference: python/ray/tune/stopper/__init__.py); the
stoppers live in ``ray_amd.tune.tuner``."""
from ray_amd.tune.tuner import (CombinedStopper, ExperimentPlateauStopper,  # noqa: F401
                                FunctionStopper, MaximumIterationStopper, NoopStopper, Stopper,
                                TimeoutStopper, TrialPlateauStopper)
