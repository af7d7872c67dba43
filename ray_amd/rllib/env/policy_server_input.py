"""``PolicyServerInput`` (reference: python/ray/rllib/env/policy_server_input.py): serve the
policy to external simulators over HTTP.

Simulators run ``PolicyClient``s (``env/policy_client.py``) in their own processes and
drive episodes through it — start_episode / get_action / log_returns / end_episode, the
``ExternalEnv`` API. The server is an ``ExternalEnv`` whose loop is an HTTP server: each
request becomes the matching ExternalEnv call, so the env runner that owns it samples the
remote episodes exactly like a local external env (observations in, the policy's actions
out, rewards credited to the step that earned them).

Use it the reference's way, as the input of an algorithm without a local env::

    config = (PPOConfig()
              .environment(env=None, observation_space=obs_space, action_space=act_space)
              .offline_data(input_=lambda ioctx: PolicyServerInput(ioctx, "127.0.0.1", 9900))
              .env_runners(num_env_runners=0))

(with ``num_env_runners=N`` each runner ``i`` serves on ``port + i - 1``). Requests and
replies are JSON (numpy arrays as typed lists); nothing is unpickled from the network.
"""

from __future__ import annotations

import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from ray_amd.rllib.env import _wire
from ray_amd.rllib.env.external_env import ExternalEnv

START_EPISODE = "START_EPISODE"
GET_ACTION = "GET_ACTION"
LOG_ACTION = "LOG_ACTION"
LOG_RETURNS = "LOG_RETURNS"
END_EPISODE = "END_EPISODE"
GET_WORKER_ARGS = "GET_WORKER_ARGS"
GET_WEIGHTS = "GET_WEIGHTS"
REPORT_SAMPLES = "REPORT_SAMPLES"


class PolicyServerInput(ExternalEnv):
    def __init__(self, ioctx=None, address: str = "127.0.0.1", port: int = 9900,
                 idle_timeout: float = 3.0, max_sample_queue_size: int = 20,
                 observation_space=None, action_space=None):
        cfg = getattr(ioctx, "config", None) or {}
        get = (cfg.get if isinstance(cfg, dict) else lambda k, d=None: getattr(cfg, k, d))
        obs = observation_space or get("observation_space")
        act = action_space or get("action_space")
        if obs is None or act is None:
            raise ValueError("PolicyServerInput needs the observation and action spaces "
                             "(AlgorithmConfig.environment(observation_space=..., "
                             "action_space=...))")
        super().__init__(act, obs)
        widx = int(getattr(ioctx, "worker_index", 0) or 0)
        self.address = address
        self.port = int(port) + max(0, widx - 1)
        self.idle_timeout = idle_timeout
        self._server = ThreadingHTTPServer((address, self.port), self._handler())
        self._server.daemon_threads = True
        self.port = self._server.server_address[1]  # port 0: an ephemeral one
        self._stopped = threading.Event()

    def _handler(self):
        ext = self

        class Handler(BaseHTTPRequestHandler):
            def log_message(self, *a):  # quiet
                pass

            def do_POST(self):
                n = int(self.headers.get("Content-Length", 0))
                try:
                    req = _wire.loads(self.rfile.read(n))
                    out = ext._execute(req)
                    code, body = 200, _wire.dumps(out)
                except Exception as e:  # noqa: BLE001 - reported to the client
                    code, body = 400, _wire.dumps({"error": f"{type(e).__name__}: {e}"})
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

        return Handler

    def _execute(self, req: dict) -> dict:
        cmd = req.get("command")
        if cmd == START_EPISODE:
            return {"episode_id": self.start_episode(req.get("episode_id"),
                                                     req.get("training_enabled", True))}
        if cmd == GET_ACTION:
            return {"action": self.get_action(req["episode_id"], req["observation"])}
        if cmd == LOG_RETURNS:
            self.log_returns(req["episode_id"], req["reward"], req.get("info"))
            return {}
        if cmd == END_EPISODE:
            self.end_episode(req["episode_id"], req["observation"])
            return {}
        if cmd == LOG_ACTION:
            self.log_action(req["episode_id"], req["observation"], req["action"])
            return {}
        if cmd in (GET_WORKER_ARGS, GET_WEIGHTS, REPORT_SAMPLES):
            raise NotImplementedError(
                "PolicyClient inference_mode='local' is not supported: use 'remote'")
        raise ValueError(f"unknown command {cmd!r}")

    def run(self):
        try:
            self._server.serve_forever(poll_interval=0.2)
        finally:
            self._stopped.set()

    def shutdown(self):
        self._server.shutdown()
        self._server.server_close()
