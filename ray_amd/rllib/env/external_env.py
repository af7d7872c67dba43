"""Externally driven environments (reference: rllib/env/external_env.py).

An ``ExternalEnv`` inverts control: the environment runs its own loop in a thread
(``run()``, written by the user, e.g. around a simulator or a service) and asks the
policy for actions::

    class Sim(ExternalEnv):
        def run(self):
            while True:
                eid = self.start_episode()
                obs = sim.reset()
                while not done:
                    a = self.get_action(eid, obs)
                    obs, r, done = sim.step(a)
                    self.log_returns(eid, r)
                self.end_episode(eid, obs)

RLlib's EnvRunners step gym-style envs, so ``make_env`` wraps an ExternalEnv in
``ExternalEnvAdapter``: ``reset()`` waits for the next episode's first observation,
``step(a)`` hands ``a`` to the blocked ``get_action`` call and returns at the next
``get_action`` (or ``end_episode``) with the rewards logged in between. The external
loop and the runner hand off through two queues, so the environment thread runs
exactly as far as the policy lets it (one action at a time, like a gym env).

Episodes of one ExternalEnv are sequential: ``start_episode`` blocks while the previous
episode is open (``max_concurrent`` is accepted for API parity; run several runners /
``num_envs_per_env_runner`` envs for concurrent episodes). Off-policy logging
(``log_action``, actions chosen outside the policy) is refused: record such data with
the offline writer (``rllib/offline``) and train with BC/MARWIL/CQL instead.
"""

from __future__ import annotations

import queue
import threading
import uuid

from ray_amd.rllib.env.envs import Env


class ExternalEnv(threading.Thread):
    def __init__(self, action_space, observation_space, max_concurrent: int = 100):
        super().__init__(daemon=True)
        self.action_space = action_space
        self.observation_space = observation_space
        self.max_concurrent = max_concurrent
        self._events: queue.Queue = queue.Queue()
        self._actions: queue.Queue = queue.Queue()
        self._episode_slot = threading.Semaphore(1)
        self._lock = threading.Lock()
        self._open: dict = {}  # episode id -> accumulated reward since the last action
        self._error = None

    def run(self):
        raise NotImplementedError("ExternalEnv subclasses implement run()")

    def _run_wrapped(self):
        try:
            self.run()
        except BaseException as e:  # noqa: BLE001 - surfaced to the runner
            self._error = e
            self._events.put(("error", None, e))

    # ------------------------------------------------------------- env-side API
    def start_episode(self, episode_id: str | None = None,
                      training_enabled: bool = True) -> str:
        self._episode_slot.acquire()
        eid = episode_id or uuid.uuid4().hex
        with self._lock:
            if eid in self._open:
                self._episode_slot.release()
                raise ValueError(f"episode {eid} is already started")
            self._open[eid] = 0.0
        return eid

    def get_action(self, episode_id: str, observation):
        self._check(episode_id)
        self._events.put(("obs", episode_id, observation))
        return self._actions.get()

    def log_action(self, episode_id: str, observation, action):
        raise NotImplementedError(
            "off-policy log_action is not sampled through EnvRunners: write the "
            "transitions with ray_amd.rllib.offline and train offline (BC/MARWIL/CQL)")

    def log_returns(self, episode_id: str, reward: float, info=None):
        with self._lock:
            self._check(episode_id)
            self._open[episode_id] += float(reward)

    def end_episode(self, episode_id: str, observation):
        self._check(episode_id)
        self._events.put(("end", episode_id, observation))
        self._episode_slot.release()

    def _check(self, eid):
        if eid not in self._open:
            raise ValueError(f"episode {eid} was not started (or already ended)")

    def _take_reward(self, eid) -> float:
        with self._lock:
            r = self._open.get(eid, 0.0)
            if eid in self._open:
                self._open[eid] = 0.0
            return r

    def _close(self, eid):
        with self._lock:
            self._open.pop(eid, None)


class ExternalEnvAdapter(Env):
    """gym-style view of an ExternalEnv (see the module docstring)."""

    def __init__(self, ext: ExternalEnv, timeout_s: float = 60.0):
        self.ext = ext
        self.observation_space = ext.observation_space
        self.action_space = ext.action_space
        self.timeout_s = timeout_s
        self._eid = None
        self._waiting = False  # the external thread is blocked in get_action
        self._thread = None  # runs ext.run() (the ExternalEnv object itself is not started)

    def _next(self):
        if not self._thread.is_alive() and self.ext._events.empty():
            raise RuntimeError("the ExternalEnv thread has exited") from self.ext._error
        try:
            ev = self.ext._events.get(timeout=self.timeout_s)
        except queue.Empty:
            raise TimeoutError(f"ExternalEnv produced no observation in {self.timeout_s}s")
        if ev[0] == "error":
            raise RuntimeError("ExternalEnv.run() raised") from ev[2]
        return ev

    def reset(self, *, seed=None, options=None):
        if self._thread is None:
            self._thread = threading.Thread(target=self.ext._run_wrapped, daemon=True,
                                            name=f"ExternalEnv-{type(self.ext).__name__}")
            self._thread.start()
        if self._eid is not None and self._waiting:
            # abandoned mid-episode (the runner reset early): finish the external side's
            # episode with the policy's default action until it ends
            while True:
                self.ext._actions.put(self.action_space.sample())
                kind, eid, obs = self._next()
                if kind == "end":
                    self.ext._close(eid)
                    break
        while True:
            kind, eid, obs = self._next()
            if kind == "obs":
                self._eid, self._waiting = eid, True
                self.ext._take_reward(eid)
                return obs, {}
            self.ext._close(eid)  # an episode that ended before asking for an action

    def step(self, action):
        if not self._waiting:
            raise RuntimeError("step() before reset()")
        self.ext._actions.put(action)
        kind, eid, obs = self._next()
        r = self.ext._take_reward(self._eid)
        if kind == "end":
            self.ext._close(eid)
            self._waiting = False
            self._eid = None
            return obs, r, True, False, {}
        return obs, r, False, False, {}


__all__ = ["ExternalEnv", "ExternalEnvAdapter"]
