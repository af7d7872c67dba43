"""ray_amd.tune — hyperparameter tuning (reference: python/ray/tune)."""

from ray_amd.air.config import CheckpointConfig, FailureConfig, RunConfig  # noqa: F401
from ray_amd.train._checkpoint import Checkpoint  # noqa: F401
from ray_amd.train._internal.session import get_checkpoint, get_context, report  # noqa: F401
from ray_amd.tune import schedulers, search  # noqa: F401
from ray_amd.tune.callback import Callback  # noqa: F401
from ray_amd.tune.logger import (CSVLogger, CSVLoggerCallback, JsonLogger,  # noqa: F401
                                 JsonLoggerCallback, LegacyLoggerCallback, Logger,
                                 LoggerCallback, NoopLogger, TBXLogger, TBXLoggerCallback,
                                 UnifiedLogger, pretty_print)
from ray_amd.tune.search.sample import (choice, grid_search, lograndint, loguniform,  # noqa
                                        qlograndint, qloguniform, qrandint, qrandn, quniform,
                                        randint, randn, sample_from, uniform)
from ray_amd.tune.trainable import Trainable, with_parameters, with_resources  # noqa: F401
from ray_amd.tune.tuner import (CombinedStopper, ExperimentAnalysis,  # noqa: F401
                                ExperimentPlateauStopper, NoopStopper,
                                FunctionStopper, MaximumIterationStopper, ResultGrid, Stopper,
                                TimeoutStopper, TrialPlateauStopper, TuneConfig, Tuner, run)
from ray_amd.train.result import Result  # noqa: F401
from ray_amd.tune.registry import (CLIReporter, Experiment,  # noqa: F401
                                   JupyterNotebookReporter, PlacementGroupFactory,
                                   ProgressReporter, create_scheduler, create_searcher,
                                   register_env, register_trainable, run_experiments)
from ray_amd.air.config import SyncConfig  # noqa: F401
from ray_amd.tune.tuner import ResumeConfig  # noqa: F401

from ray_amd.tune.error import TuneError  # noqa: E402,F401


