"""reference: python/ray/tune/experiment/__init__.py."""

from ray_amd.tune.registry import Experiment  # noqa: F401
from ray_amd.tune.tuner import Trial  # noqa: F401


def _convert_to_experiment_list(experiments):
    """A single Experiment, a list of them, or a ``{name: spec}`` dict -> a list."""
    if experiments is None:
        return []
    if isinstance(experiments, Experiment):
        return [experiments]
    if isinstance(experiments, dict):
        return [e if isinstance(e, Experiment) else Experiment(name, **e)
                for name, e in experiments.items()]
    if isinstance(experiments, (list, tuple)):
        if not all(isinstance(e, Experiment) for e in experiments):
            raise TypeError("experiments must be Experiment objects")
        return list(experiments)
    raise TypeError(f"invalid experiments: {type(experiments).__name__}")


__all__ = ["Experiment", "_convert_to_experiment_list", "Trial"]
