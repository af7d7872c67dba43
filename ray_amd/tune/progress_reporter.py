"""``ray.tune.progress_reporter`` (reference: python/ray/tune/progress_reporter.py)."""

from ray_amd.tune.registry import (CLIReporter, JupyterNotebookReporter,  # noqa: F401
                                   ProgressReporter)

TuneReporterBase = CLIReporter


class RemoteReporterMixin:
    """Reporters whose output is shown somewhere else than the driver's stdout: output
    goes to ``output_queue`` when one is set."""

    @property
    def output_queue(self):
        return getattr(self, "_output_queue", None)

    @output_queue.setter
    def output_queue(self, value):
        self._output_queue = value

    def display(self, string: str) -> None:
        q = self.output_queue
        if q is not None:
            q.put(string)
        else:
            print(string, flush=True)


__all__ = ["ProgressReporter", "CLIReporter", "JupyterNotebookReporter", "TuneReporterBase",
           "RemoteReporterMixin"]
