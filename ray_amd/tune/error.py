"""``ray.tune.error`` (reference: python/ray/tune/error.py)."""


class TuneError(RuntimeError):
    """A Tune experiment failed; tune.run raises it when trials errored and
    raise_on_failed_trial is left True."""


class _AbortTrialExecution(TuneError):
    """Abort a trial's execution (an unrecoverable setup error)."""


class _SubCategoryTuneError(TuneError):
    """A TuneError carrying the original exception as ``traceback_str``."""

    def __init__(self, traceback_str: str = ""):
        self.traceback_str = traceback_str
        super().__init__(traceback_str)
