"""The policy server's shared-memory mailbox protocol on CPU (rllib/env/policy_server.py):
runner slots in REQUEST are gathered, answered with RESPONSE and read back by their own
client, from several client processes at once. The GPU forward itself is covered by
tests/test_rllib_gpu_runner.py::test_policy_server_serves_all_runners."""
import mmap
import multiprocessing as mp
import os
import threading
import time

import numpy as np

from ray_amd._private import shm_segment
from ray_amd.rllib.env.policy_server import IDLE, REQUEST, RESPONSE, PolicyClient, _Layout


class _FakeServer:
    """The server's gather/answer loop with a numpy 'policy': logits = first pixels."""

    def __init__(self, n_slots, B, shape, n):
        self.lay = _Layout(n_slots, B, shape, n)
        self.path, self.fd = shm_segment.create("ramd_polsrv_test")
        os.ftruncate(self.fd, self.lay.size)
        self.mm = mmap.mmap(self.fd, self.lay.size)
        self.state, self.obs, self.u, self.out = self.lay.views(self.mm)
        self.state[:] = IDLE
        self.stop = False
        self.batches = 0
        self.t = threading.Thread(target=self.loop, daemon=True)
        self.t.start()

    def loop(self):
        n = self.lay.n
        while not self.stop:
            ready = np.flatnonzero(self.state == REQUEST)
            if len(ready) == 0:
                time.sleep(0.0001)
                continue
            for s in ready:
                logits = self.obs[s][:, 0, 0, :n].astype(np.float32)
                explore = self.u[s][:, n]
                a = np.where(explore > 0, np.argmax(self.u[s][:, :n], 1), np.argmax(logits, 1))
                self.out[s][:, 0] = a
                self.out[s][:, 1] = -1.0
                self.out[s][:, 2:] = logits
            self.state[ready] = RESPONSE
            self.batches += 1


def _client_proc(path, slot, n_slots, B, shape, n, q):
    c = PolicyClient(path, slot, n_slots, B, shape, n)
    rng = np.random.default_rng(slot)
    ok = True
    for i in range(200):
        obs = np.zeros((B,) + shape, np.uint8)
        obs[:, 0, 0, :n] = rng.integers(0, 200, (B, n))
        a, lp, di = c.step(obs, False, rng)
        ok &= bool(np.array_equal(a, np.argmax(obs[:, 0, 0, :n], 1)))
        ok &= bool(np.array_equal(di, obs[:, 0, 0, :n].astype(np.float32)))
    q.put((slot, ok))


def test_mailbox_round_trips_from_many_clients():
    shape, n, B, slots = (8, 8, 6), 6, 3, 4
    srv = _FakeServer(slots, B, shape, n)
    try:
        ctx = mp.get_context("fork")
        q = ctx.Queue()
        ps = [ctx.Process(target=_client_proc, args=(srv.path, s, slots, B, shape, n, q))
              for s in range(slots)]
        for p in ps:
            p.start()
        res = dict(q.get(timeout=60) for _ in ps)
        for p in ps:
            p.join(timeout=10)
        assert res == {s: True for s in range(slots)}
        assert srv.batches >= 200  # batched: at most one answer per slot per round
        # explore: the draw comes from the client's uniforms (Gumbel input) per row
        c = PolicyClient(srv.path, 0, slots, B, shape, n)
        a, _, _ = c.step(np.zeros((B,) + shape, np.uint8), True, np.random.default_rng(3))
        u = np.random.default_rng(3).random((B, n))
        assert np.array_equal(a, np.argmax(u, 1))
    finally:
        srv.stop = True
        srv.t.join(timeout=2)
        shm_segment.release(srv.path, srv.fd)
