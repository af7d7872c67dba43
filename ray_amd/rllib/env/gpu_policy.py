"""Env-runner policy inference on the MI355X as one HIP graph per step.

The reference's env runners run their RLModule wherever ``num_gpus_per_env_runner`` puts
it (rllib/env/single_agent_env_runner.py: ``_sample`` → ``forward_exploration`` on the
module's device) and pay one eager launch per op plus the host round trips. At the Atari
PPO shape (5 envs per runner) that launch and sync overhead is larger than the Nature-CNN
itself, so here the whole step is captured once:

    pinned obs / uniforms ──H2D──▶ conv.hip MFMA convs (uint8 frames read directly, /255
    fused) ─▶ FC ─▶ logits ─▶ log-softmax, Gumbel-max draw, log-prob ─▶ [a | logp | logits]
    ──D2H──▶ pinned output

and every step is: two host memcpys into pinned staging, ``graph.replay()``, one stream
sync. The uniforms come from the runner's numpy generator (seeded like the CPU path), so
the sampling is reproducible and a CPU module given the same uniforms draws the same
actions (tests/test_rllib_gpu_runner.py). Weights are updated in place
(``load_state_dict`` copies into the captured parameter storage), so a new policy version
needs no re-capture. A runner process also caps its HIP hardware queues (one stream is all
it uses): 8 runners x 8 queues next to the learner oversubscribe the queue slots.
"""

from __future__ import annotations

import numpy as np
import torch


class GraphedDiscretePolicy:
    """Categorical policy step of an actor-critic RLModule, replayed as a HIP graph.

    ``step(obs, explore, rng)`` returns ``(actions int64 [B], logp [B], dist_inputs [B, n])``
    as numpy arrays (views of pinned memory, valid until the next step)."""

    def __init__(self, module, obs_example: np.ndarray, n_actions: int, device):
        self.module = module
        self.device = torch.device(device)
        self.B = obs_example.shape[0]
        self.obs_shape = tuple(obs_example.shape)
        self.obs_dtype = obs_example.dtype
        self.n = int(n_actions)
        tdt = torch.from_numpy(np.empty(0, self.obs_dtype)).dtype
        self.obs_pin = torch.empty(self.obs_shape, dtype=tdt).pin_memory()
        # uniforms for the Gumbel draw; the last column is the explore flag (0 / 1)
        self.u_pin = torch.empty((self.B, self.n + 1), dtype=torch.float32).pin_memory()
        self.out_pin = torch.empty((self.B, 2 + self.n), dtype=torch.float32).pin_memory()
        self.obs_np = self.obs_pin.numpy()
        self.u_np = self.u_pin.numpy()
        self.out_np = self.out_pin.numpy()
        self.obs_dev = torch.empty(self.obs_shape, dtype=tdt, device=self.device)
        self.u_dev = torch.empty((self.B, self.n + 1), dtype=torch.float32, device=self.device)
        self.out_dev = torch.empty((self.B, 2 + self.n), dtype=torch.float32, device=self.device)
        self.graph = None
        self._capture()

    def _body(self):
        self.obs_dev.copy_(self.obs_pin, non_blocking=True)
        self.u_dev.copy_(self.u_pin, non_blocking=True)
        di = self.module.forward_inference(self.obs_dev)["action_dist_inputs"].float()
        lp = torch.log_softmax(di, -1)
        u = self.u_dev[:, :self.n].clamp(1e-20, 1.0)
        g = -torch.log(-torch.log(u)) * self.u_dev[:, self.n:]
        a = (lp + g).argmax(-1)
        logp = lp.gather(-1, a[:, None])
        torch.cat([a.float()[:, None], logp, di], 1, out=self.out_dev)
        self.out_pin.copy_(self.out_dev, non_blocking=True)

    def _capture(self):
        self.obs_np[...] = 0
        self.u_np[...] = 0.5
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.no_grad(), torch.cuda.stream(side):
            for _ in range(2):  # allocator / kernel warmup outside the capture
                self._body()
        torch.cuda.current_stream(self.device).wait_stream(side)
        torch.cuda.synchronize(self.device)
        from ray_amd.ops.graph_lock import CAPTURE_LOCK

        g = torch.cuda.CUDAGraph()
        with CAPTURE_LOCK, torch.no_grad(), torch.cuda.graph(g):
            self._body()
        self.graph = g

    def step(self, obs: np.ndarray, explore: bool, rng: np.random.Generator):
        np.copyto(self.obs_np, obs, casting="unsafe")
        if explore:
            self.u_np[:, :self.n] = rng.random((self.B, self.n))
            self.u_np[:, self.n] = 1.0
        else:
            self.u_np[:, self.n] = 0.0
            self.u_np[:, :self.n] = 0.5
        from ray_amd.ops.graph_lock import CAPTURE_LOCK

        with CAPTURE_LOCK:
            self.graph.replay()
            torch.cuda.current_stream(self.device).synchronize()
        h = self.out_np
        return h[:, 0].astype(np.int64), h[:, 1], h[:, 2:]


def cpu_reference_step(module, obs: np.ndarray, u: np.ndarray, explore: bool):
    """The same step on a CPU module with given uniforms [B, n] (tests: GPU vs CPU)."""
    with torch.no_grad():
        di = module.forward_inference(torch.from_numpy(obs))["action_dist_inputs"].float()
        lp = torch.log_softmax(di, -1)
        if explore:
            g = -torch.log(-torch.log(torch.from_numpy(u).clamp(1e-20, 1.0)))
            a = (lp + g).argmax(-1)
        else:
            a = lp.argmax(-1)
        logp = lp.gather(-1, a[:, None])[:, 0]
    return a.numpy(), logp.numpy(), di.numpy()
