"""Tune callbacks: experiment-level hooks run on the driver.

API contract (reference: python/ray/tune/callback.py:70 ``Callback`` —
``setup``, ``on_step_begin``, ``on_step_end``, ``on_trial_start``,
``on_trial_restore``, ``on_trial_save``, ``on_trial_result``, ``on_trial_complete``,
``on_trial_error``, ``on_checkpoint``, ``on_experiment_end``; every hook takes
``iteration``, ``trials``, ``trial`` and ``**info``).

Design: the controller owns one ``CallbackList`` and fires each event once; a
callback that raises is reported and disabled instead of killing the experiment.
Trainers (DataParallelTrainer.fit) fire the same events for their single pseudo-trial,
so ``RunConfig(callbacks=[...])`` behaves the same under Tuner and Trainer.
"""

from __future__ import annotations

import sys
import traceback


class Callback:
    """Base class: override any subset of hooks."""

    def setup(self, stop=None, num_samples=None, total_num_samples=None, **info):
        pass

    def on_step_begin(self, iteration: int, trials: list, **info):
        pass

    def on_step_end(self, iteration: int, trials: list, **info):
        pass

    def on_trial_start(self, iteration: int, trials: list, trial, **info):
        pass

    def on_trial_restore(self, iteration: int, trials: list, trial, **info):
        pass

    def on_trial_save(self, iteration: int, trials: list, trial, **info):
        pass

    def on_trial_result(self, iteration: int, trials: list, trial, result: dict, **info):
        pass

    def on_trial_complete(self, iteration: int, trials: list, trial, **info):
        pass

    def on_trial_recover(self, iteration: int, trials: list, trial, **info):
        pass

    def on_trial_error(self, iteration: int, trials: list, trial, **info):
        pass

    def on_checkpoint(self, iteration: int, trials: list, trial, checkpoint, **info):
        pass

    def on_experiment_end(self, trials: list, **info):
        pass

    # experiment-state persistence hooks (reference: Callback.get_state / set_state)
    def get_state(self):
        return None

    def set_state(self, state):
        pass


class CallbackList:
    def __init__(self, callbacks):
        self.callbacks = [c for c in (callbacks or []) if c is not None]
        self.iteration = 0

    def __len__(self):
        return len(self.callbacks)

    def fire(self, hook: str, **kw):
        for cb in list(self.callbacks):
            fn = getattr(cb, hook, None)
            if fn is None:
                continue
            try:
                if hook in ("setup", "on_experiment_end"):
                    fn(**kw)
                else:
                    fn(iteration=self.iteration, **kw)
            except Exception:  # noqa: BLE001
                print(f"[ray_amd.tune] callback {type(cb).__name__}.{hook} raised; disabling "
                      f"it:\n{traceback.format_exc()}", file=sys.stderr, flush=True)
                self.callbacks.remove(cb)

    def step(self, trials):
        self.iteration += 1
        self.fire("on_step_begin", trials=trials)

    def end_step(self, trials):
        self.fire("on_step_end", trials=trials)
