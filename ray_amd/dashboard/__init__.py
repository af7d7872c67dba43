"""HTTP head (state / metrics / jobs REST) — see ``head.py``.

``start_dashboard(session_dir, port)`` launches it as a child process of the caller
and waits until it serves.
"""

from __future__ import annotations

import json
import os
import subprocess
import sys
import time


def start_dashboard(session_dir: str, host: str = "127.0.0.1", port: int = 8265,
                    timeout: float = 60.0):
    url_file = os.path.join(session_dir, "dashboard.json")
    try:
        os.unlink(url_file)
    except FileNotFoundError:
        pass
    env = dict(os.environ)
    pkg_root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env["PYTHONPATH"] = pkg_root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH")
                                    else "")
    env.pop("RAY_ADDRESS", None)
    log = open(os.path.join(session_dir, "dashboard.log"), "ab")
    proc = subprocess.Popen([sys.executable, "-m", "ray_amd.dashboard.head", "--session-dir",
                             session_dir, "--host", host, "--port", str(port)], env=env,
                            stdout=log, stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL,
                            start_new_session=True)
    t0 = time.time()
    while not os.path.exists(url_file):
        if proc.poll() is not None:
            raise RuntimeError(f"dashboard exited with code {proc.returncode}; see "
                               f"{os.path.join(session_dir, 'dashboard.log')}")
        if time.time() - t0 > timeout:
            proc.kill()
            raise RuntimeError("timed out waiting for the dashboard")
        time.sleep(0.05)
    with open(url_file) as f:
        info = json.load(f)
    return proc, info["url"]
