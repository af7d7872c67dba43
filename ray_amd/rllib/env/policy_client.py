"""``PolicyClient`` (reference: python/ray/rllib/env/policy_client.py): the simulator side
of ``PolicyServerInput`` — ExternalEnv-style calls sent over HTTP as JSON.

Only ``inference_mode="remote"`` is supported: every ``get_action`` is answered by the
server's env runner with the current policy (no local copy of the model in the client)."""

from __future__ import annotations

import time
import urllib.error
import urllib.request
from typing import Optional

from ray_amd.rllib.env import _wire
from ray_amd.rllib.env.policy_server_input import (END_EPISODE, GET_ACTION, LOG_ACTION,
                                                   LOG_RETURNS, START_EPISODE)


class PolicyClient:
    def __init__(self, address: str, inference_mode: str = "remote",
                 update_interval: float = 10.0, session=None, connect_timeout_s: float = 60.0,
                 request_timeout_s: float = 300.0):
        if inference_mode != "remote":
            raise NotImplementedError("PolicyClient supports inference_mode='remote' only")
        self.address = address if address.startswith("http") else f"http://{address}"
        self.inference_mode = inference_mode
        self.connect_timeout_s = connect_timeout_s
        self.request_timeout_s = request_timeout_s

    def _send(self, data: dict) -> dict:
        body = _wire.dumps(data)
        t0 = time.monotonic()
        while True:
            req = urllib.request.Request(self.address, data=body, method="POST",
                                         headers={"Content-Type": "application/json"})
            try:
                with urllib.request.urlopen(req, timeout=self.request_timeout_s) as r:
                    return _wire.loads(r.read())
            except urllib.error.HTTPError as e:
                msg = _wire.loads(e.read()).get("error", str(e))
                raise RuntimeError(f"policy server error: {msg}") from None
            except (urllib.error.URLError, ConnectionError) as e:
                # the server binds when its env runner starts: retry until it is up
                if time.monotonic() - t0 > self.connect_timeout_s:
                    raise ConnectionError(f"policy server {self.address} unreachable") from e
                time.sleep(0.2)

    def start_episode(self, episode_id: Optional[str] = None,
                      training_enabled: bool = True) -> str:
        return self._send({"command": START_EPISODE, "episode_id": episode_id,
                           "training_enabled": training_enabled})["episode_id"]

    def get_action(self, episode_id: str, observation):
        return self._send({"command": GET_ACTION, "episode_id": episode_id,
                           "observation": observation})["action"]

    def log_action(self, episode_id: str, observation, action) -> None:
        self._send({"command": LOG_ACTION, "episode_id": episode_id,
                    "observation": observation, "action": action})

    def log_returns(self, episode_id: str, reward, info=None,
                    multiagent_done_dict=None) -> None:
        self._send({"command": LOG_RETURNS, "episode_id": episode_id,
                    "reward": float(reward), "info": info})

    def end_episode(self, episode_id: str, observation) -> None:
        self._send({"command": END_EPISODE, "episode_id": episode_id,
                    "observation": observation})

    def update_policy_weights(self) -> None:
        """Remote inference uses the server's current weights: nothing to fetch."""
