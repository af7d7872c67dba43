"""A node started by ray.init() shares the driver's fate (reference: services.py
start_ray_process(fate_share=True)): a driver killed without ray.shutdown() leaves no
raylet, no workers and no /dev/shm object-store file behind."""

import json
import os
import subprocess
import sys
import textwrap
import time


def _alive(pid):
    try:
        os.kill(pid, 0)
        return True
    except ProcessLookupError:
        return False


def test_killed_driver_takes_its_node_down(tmp_path):
    out = tmp_path / "info.json"
    code = textwrap.dedent(f"""
        import json, os
        import ray_amd as ray
        ray.init(num_cpus=1)
        @ray.remote
        def pid():
            return os.getpid()
        w = ray.get(pid.remote())
        from ray_amd._private.worker import global_worker
        cw = global_worker.core
        sess = global_worker.session_dir if hasattr(global_worker, "session_dir") else None
        info = {{"worker": w, "store": cw.cluster_info.get("store_path")}}
        with open({str(out)!r}, "w") as f:
            json.dump(info, f)
        os._exit(0)  # no ray.shutdown(), no atexit
    """)
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=repo + os.pathsep + os.environ.get("PYTHONPATH", ""))
    before = set(os.listdir("/dev/shm"))
    subprocess.run([sys.executable, "-c", code], env=env, timeout=120, check=True)
    info = json.loads(out.read_text())
    deadline = time.time() + 20
    while time.time() < deadline and _alive(info["worker"]):
        time.sleep(0.2)
    assert not _alive(info["worker"])
    store = info.get("store")
    if store:
        while time.time() < deadline and os.path.exists(store):
            time.sleep(0.2)
        assert not os.path.exists(store)
    leaked = [f for f in set(os.listdir("/dev/shm")) - before if f.startswith("ray_amd_session")]
    assert not leaked
