"""One batched policy-inference process on the MI355X for all env runners.

Reference: RLlib's env runners each run their RLModule where ``num_gpus_per_env_runner``
puts it (rllib/env/single_agent_env_runner.py ``_sample``). Eight runner processes each
driving the GPU for a 5-frame Nature-CNN forward per step time-share the device with the
learner (profiles/r6/README.md: 26k env-steps/s against 71k with CPU inference). Here the
runners keep stepping their envs on CPU and hand the policy forward to ONE process that
owns the GPU work:

* a shared-memory mailbox (an anonymous memfd of the server, opened by the runners
  through ``/proc/<pid>/fd``) holds one slot per runner: uint8 frames in, the Gumbel
  uniforms, and ``[action | logp | logits]`` out, plus a per-slot state word;
* the server thread gathers every slot in state REQUEST, copies them into one pinned batch
  (all runners x envs rows), replays ONE captured HIP graph (``GraphedDiscretePolicy``:
  conv.hip MFMA convolutions on the uint8 frames, log-softmax, Gumbel-max draw), and
  writes each slot's rows back with state RESPONSE;
* a runner spins on its own state word (it has nothing else to do in the meantime), so a
  step costs one memcpy each way plus the batched forward, with no RPC and no GPU context
  in the runner.

With a local learner (``num_learners=0``) the server is a thread of the learner's own
process: one GPU context, the forward passes on their own stream beside the learner's
kernels, HIP-graph captures serialized through ``ops.graph_lock``. With remote learners it
is an actor holding ``num_gpus_per_policy_server`` of a GPU.

Weights reach the server through ``set_weights`` beside the runners' weight sync. The
uniforms are drawn by each runner from its own generator, so the actions are the same as
the runner's local GPU graph path would draw for the same weights.
"""

from __future__ import annotations

import mmap
import os
import threading
import time

import numpy as np

IDLE, REQUEST, RESPONSE = 0, 1, 2
_LINE = 64  # one cache line per slot state word


def _round(n, a=4096):
    return (n + a - 1) // a * a


class _Layout:
    def __init__(self, n_slots, B, obs_shape, n_actions):
        self.n_slots, self.B, self.n = int(n_slots), int(B), int(n_actions)
        self.obs_shape = tuple(int(x) for x in obs_shape)
        self.obs_bytes = self.B * int(np.prod(self.obs_shape))
        self.u_bytes = self.B * (self.n + 1) * 4
        self.out_bytes = self.B * (2 + self.n) * 4
        self.slot_bytes = _round(self.obs_bytes + self.u_bytes + self.out_bytes)
        self.head = _round(self.n_slots * _LINE)
        self.size = self.head + self.n_slots * self.slot_bytes

    def views(self, buf):
        st = np.frombuffer(buf, np.int32, self.n_slots * _LINE // 4, 0)[::_LINE // 4]
        obs, u, out = [], [], []
        for s in range(self.n_slots):
            o = self.head + s * self.slot_bytes
            obs.append(np.frombuffer(buf, np.uint8, self.obs_bytes, o).reshape(
                (self.B,) + self.obs_shape))
            u.append(np.frombuffer(buf, np.float32, self.u_bytes // 4,
                                   o + self.obs_bytes).reshape(self.B, self.n + 1))
            out.append(np.frombuffer(buf, np.float32, self.out_bytes // 4,
                                     o + self.obs_bytes + self.u_bytes).reshape(
                self.B, 2 + self.n))
        return st, obs, u, out


class PolicyServer:
    """In-process server or actor body (``ray.remote(num_gpus=...)(PolicyServer)``):
    ``module_fn`` builds the RLModule; the mailbox has ``n_slots`` slots of ``B`` envs."""

    def __init__(self, module_fn, n_slots, B, obs_shape, n_actions):
        import torch

        from ray_amd._private import shm_segment

        self.lay = _Layout(n_slots, B, obs_shape, n_actions)
        self.path, self._fd = shm_segment.create(f"ramd_polsrv_{os.getpid()}")
        os.ftruncate(self._fd, self.lay.size)
        self._mm = mmap.mmap(self._fd, self.lay.size)
        self.state, self.obs, self.u, self.out = self.lay.views(self._mm)
        self.state[:] = IDLE
        self.device = torch.device("cuda", 0)
        self.module = module_fn().to(self.device)
        if getattr(self.module, "is_image", False):
            self.module.to(torch.bfloat16).to(memory_format=torch.channels_last)
        self.module.eval()
        from ray_amd.rllib.env.gpu_policy import GraphedDiscretePolicy

        total = self.lay.n_slots * self.lay.B
        self.pol = GraphedDiscretePolicy(
            self.module, np.zeros((total,) + self.lay.obs_shape, np.uint8), self.lay.n,
            self.device)
        self._lock = threading.Lock()
        self._stop = False
        self.batches = 0
        self.rows = 0
        self.version = -1
        self._t = threading.Thread(target=self._loop, name="policy-server", daemon=True)
        self._t.start()

    def mailbox(self):
        return self.path, self.lay.n_slots, self.lay.B, self.lay.obs_shape, self.lay.n

    def set_weights(self, weights, version=None):
        import torch

        if version is not None and version == self.version:
            return
        w = {k: v for k, v in dict(weights).items() if not k.startswith("__")}
        sd = {k: (v if isinstance(v, torch.Tensor) else torch.as_tensor(v))
              for k, v in w.items()}
        with self._lock:  # copies into the captured parameter storage
            self.module.load_state_dict(sd)
            torch.cuda.current_stream(self.device).synchronize()
        self.version = version if version is not None else self.version

    def stats(self):
        return {"batches": self.batches, "rows": self.rows}

    def _loop(self):
        import torch

        from ray_amd.ops.graph_lock import CAPTURE_LOCK

        B, n = self.lay.B, self.lay.n
        pol = self.pol
        # its own stream: in the learner's process the forward passes overlap the
        # learner's kernels instead of queueing behind them
        torch.cuda.set_stream(torch.cuda.Stream(self.device))
        idle_spins = 0
        while not self._stop:
            ready = np.flatnonzero(self.state == REQUEST)
            if len(ready) == 0:
                idle_spins += 1
                if idle_spins > 2000:  # nobody sampling: back off
                    time.sleep(0.0005)
                continue
            idle_spins = 0
            with self._lock:
                # gather the ready slots into the batch's leading rows (the rest keep
                # whatever they held: their outputs are not read)
                for j, s in enumerate(ready):
                    pol.obs_np[j * B:(j + 1) * B] = self.obs[s]
                    pol.u_np[j * B:(j + 1) * B] = self.u[s]
                with CAPTURE_LOCK:
                    pol.graph.replay()
                    torch.cuda.current_stream(self.device).synchronize()
                for j, s in enumerate(ready):
                    self.out[s][...] = pol.out_np[j * B:(j + 1) * B]
            self.state[ready] = RESPONSE
            self.batches += 1
            self.rows += len(ready) * B

    def shutdown(self):
        self._stop = True
        self._t.join(timeout=2)


class PolicyClient:
    """A runner's view of one mailbox slot."""

    def __init__(self, path, slot, n_slots, B, obs_shape, n_actions):
        self.lay = _Layout(n_slots, B, obs_shape, n_actions)
        fd = os.open(path, os.O_RDWR)
        try:
            self._mm = mmap.mmap(fd, self.lay.size)
        finally:
            os.close(fd)
        st, obs, u, out = self.lay.views(self._mm)
        self.slot = int(slot)
        self.state, self.obs, self.u, self.out = st, obs[slot], u[slot], out[slot]
        self.n = self.lay.n
        self.B = self.lay.B

    def step(self, obs, explore, rng, timeout=30.0):
        """Same contract as ``GraphedDiscretePolicy.step``."""
        np.copyto(self.obs, obs, casting="unsafe")
        if explore:
            self.u[:, :self.n] = rng.random((self.B, self.n))
            self.u[:, self.n] = 1.0
        else:
            self.u[:, :self.n] = 0.5
            self.u[:, self.n] = 0.0
        st = self.state
        s = self.slot
        st[s] = REQUEST
        t0 = time.monotonic()
        spins = 0
        while st[s] != RESPONSE:
            spins += 1
            if spins > 20000:
                time.sleep(0.00005)
                if time.monotonic() - t0 > timeout:
                    raise TimeoutError("policy server did not answer")
        h = self.out.copy()
        st[s] = IDLE
        return h[:, 0].astype(np.int64), h[:, 1], h[:, 2:]
