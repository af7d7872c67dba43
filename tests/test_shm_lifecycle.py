"""Object-store and channel segments cannot outlive their processes (reference: plasma
unlinks its arena right after mapping it, src/ray/object_manager/plasma/dlmalloc.cc:
143,162-165). Here they are memfds opened through /proc/<owner>/fd (shm_segment.py)."""

import os
import signal
import subprocess
import sys
import time

import numpy as np

import ray_amd as ray
from ray_amd._private import shm_segment
from ray_amd.cluster_utils import Cluster


def _shm():
    return set(os.listdir("/dev/shm"))


@ray.remote
def big(n):
    return np.ones(n, dtype=np.uint8)


def test_cluster_with_killed_node_leaves_dev_shm_unchanged():
    before = _shm()
    c = Cluster(initialize_head=True, head_node_args={"num_cpus": 1})
    n1 = c.add_node(num_cpus=1, resources={"a": 1})
    n2 = c.add_node(num_cpus=1, resources={"b": 1})
    ray.init(address=c.address)
    try:
        stores = {n["NodeID"]: n["ObjectStoreSocketName"] for n in ray.nodes()}
        assert all(shm_segment.is_anonymous(p) for p in stores.values()), stores
        assert all(os.path.exists(p) for p in stores.values())
        # objects in every store (one per node)
        refs = [big.options(resources={"a": 1}).remote(1 << 20),
                big.options(resources={"b": 1}).remote(1 << 20), ray.put(np.ones(1 << 20))]
        assert [int(np.asarray(ray.get(r)).sum()) for r in refs] == [1 << 20] * 3
        assert _shm() == before  # nothing is ever named in /dev/shm
        os.kill(n1.proc.pid, signal.SIGKILL)  # a crashed node agent
        n1.proc.wait(timeout=10)
        deadline = time.time() + 10
        while time.time() < deadline and os.path.exists(stores[n1.node_id]):
            time.sleep(0.1)
        assert not os.path.exists(stores[n1.node_id])
    finally:
        ray.shutdown()
        c.shutdown()
    assert not n2.alive()
    assert _shm() == before
    for p in stores.values():
        assert not os.path.exists(p)


def test_sweep_removes_named_segments_of_dead_creators(tmp_path):
    d = tmp_path / "shm"
    d.mkdir()
    p = subprocess.Popen([sys.executable, "-c", "pass"])
    p.wait()
    dead, live = p.pid, os.getpid()
    names = [f"ray_amd_session_2026-01-01_00-00-00_{dead}_abc123",
             f"ray_amd_session_2026-01-01_00-00-00_{dead}_abc123_n2",
             f"ramd_ch_{dead}_0123456789abcdef.r1",
             f"ray_amd_session_2026-01-01_00-00-00_{live}_abc123",
             f"ramd_ch_{live}_0123456789abcdef", "unrelated_file"]
    for n in names:
        (d / n).write_bytes(b"x")
    removed = shm_segment.sweep_dead(str(d))
    assert sorted(removed) == sorted(names[:3])
    assert sorted(os.listdir(d)) == sorted(names[3:])


def test_channel_segments_are_anonymous_and_follow_resize():
    from ray_amd.experimental.channel import Channel

    before = _shm()
    ch = Channel(1, 64)
    assert shm_segment.is_anonymous(ch.path)
    rd = Channel(1, _path=ch.path)  # a reader endpoint attached by path
    ch.write(b"y" * 1000)  # grows past the 64-byte buffer
    assert rd.read() == b"y" * 1000
    ch.write("small")
    assert rd.read() == "small"
    assert _shm() == before
    paths = [p for p, _ in ch._created]
    ch.destroy()
    assert not any(os.path.exists(p) for p in paths)
