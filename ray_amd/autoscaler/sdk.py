"""Programmatic autoscaler requests (reference: python/ray/autoscaler/sdk/sdk.py
request_resources)."""

from __future__ import annotations

import pickle


def request_resources(num_cpus: int | None = None, bundles: list | None = None) -> None:
    """Ask the autoscaler to scale to fit `num_cpus` CPUs and/or `bundles` immediately,
    regardless of task demand. A later call replaces the request; ``request_resources()``
    with no arguments clears it."""
    from ray_amd._private import worker as W

    req = []
    if num_cpus:
        req.extend({"CPU": 1.0} for _ in range(int(num_cpus)))
    for b in bundles or []:
        req.append({k: float(v) for k, v in b.items()})
    W.global_worker.core.call_raylet("kv_put", "__autoscaler", b"resource_request",
                                     pickle.dumps(req), True)


# ------------------------------------------------------------------ cluster launcher
# reference: python/ray/autoscaler/sdk/sdk.py (create_or_update_cluster, teardown_cluster,
# run_on_cluster, rsync, get_head_node_ip, ...) over autoscaler/_private/commands.py.
# Provider here: "local" — every node of the cluster YAML is a process on this machine
# (head raylet + one node agent per worker), the same processes `start` launches; the
# cloud providers of the reference need their SDKs and credentials and are refused.
import copy as _copy
import json as _json
import logging as _logging
import os as _os
import shutil as _shutil
import subprocess as _subprocess
import sys as _sys
import time as _time

_CALLBACKS: dict = {}
_STATE_DIR = _os.environ.get("RAY_AMD_CLUSTER_STATE_DIR") or \
    _os.path.join(_os.path.expanduser("~"), ".ray_amd", "clusters")

_DEFAULTS = {
    "cluster_name": "default",
    "max_workers": 2,
    "upscaling_speed": 1.0,
    "idle_timeout_minutes": 5,
    "provider": {"type": "local"},
    "available_node_types": {
        "head": {"resources": {"CPU": 1}, "node_config": {}, "max_workers": 0},
        "worker": {"resources": {"CPU": 1}, "node_config": {}, "min_workers": 0,
                   "max_workers": 2},
    },
    "head_node_type": "head",
    "file_mounts": {},
    "initialization_commands": [],
    "setup_commands": [],
    "head_setup_commands": [],
    "worker_setup_commands": [],
    "head_start_ray_commands": [],
    "worker_start_ray_commands": [],
}


def _load(cluster_config):
    if isinstance(cluster_config, dict):
        return _copy.deepcopy(cluster_config)
    import yaml

    with open(_os.path.expanduser(cluster_config)) as f:
        return yaml.safe_load(f) or {}


def fillout_defaults(config: dict) -> dict:
    """The config with every launcher default filled in (reference: fillout_defaults)."""
    out = _copy.deepcopy(_DEFAULTS)
    for k, v in (config or {}).items():
        if isinstance(v, dict) and isinstance(out.get(k), dict) and k != "available_node_types":
            out[k].update(v)
        else:
            out[k] = _copy.deepcopy(v)
    return out


def bootstrap_config(config: dict, no_config_cache: bool = False) -> dict:
    """Validate and complete a cluster config for its provider."""
    cfg = fillout_defaults(_load(config))
    ptype = cfg["provider"].get("type", "local")
    if ptype != "local":
        raise ValueError(f"provider type {ptype!r} needs its cloud SDK and credentials; this "
                         "launcher runs the 'local' provider (all nodes on this machine)")
    types = cfg["available_node_types"]
    if cfg["head_node_type"] not in types:
        raise ValueError(f"head_node_type {cfg['head_node_type']!r} is not in "
                         f"available_node_types {sorted(types)}")
    return cfg


def register_callback_handler(event_name: str, callback) -> None:
    """Call ``callback(event_data)`` at launcher events ("up_started", "head_started",
    "worker_started", "up_completed", "down_completed")."""
    _CALLBACKS.setdefault(event_name, []).append(callback)


def _fire(event, data):
    for cb in _CALLBACKS.get(event, []):
        cb(data)


def configure_logging(log_style: str | None = None, color_mode: str | None = None,
                      verbosity: int | None = None) -> None:
    level = _logging.DEBUG if (verbosity or 0) > 0 else _logging.INFO
    _logging.getLogger("ray_amd.autoscaler").setLevel(level)


def get_docker_host_mount_location(cluster_name: str) -> str:
    return f"/tmp/ray_docker_mounts/{cluster_name}"


def _state_file(name):
    return _os.path.join(_STATE_DIR, f"{name}.json")


def _read_state(name):
    try:
        with open(_state_file(name)) as f:
            return _json.load(f)
    except FileNotFoundError:
        return None


def _alive(pid):
    try:
        _os.kill(pid, 0)
        return True
    except ProcessLookupError:
        return False
    except PermissionError:
        return True


def _run_cmds(cmds, env=None):
    for c in cmds or []:
        _subprocess.run(c, shell=True, check=True, env=env)


def _start_node(session, ntype, spec, head_sock):
    res = dict(spec.get("resources") or {})
    ncpu = res.pop("CPU", None)
    ngpu = res.pop("GPU", None)
    tag = _os.urandom(4).hex()
    ready = f"node_{tag}.ready"
    cmd = [_sys.executable, "-m", "ray_amd._private.raylet", "--session-dir", session,
           "--store-path", f"/dev/shm/ray_amd_{_os.path.basename(session)}_{tag}",
           "--object-store-memory", str(int(spec.get("object_store_memory", 256 << 20))),
           "--resources", _json.dumps(res), "--labels",
           _json.dumps({"ray.io/node-type": ntype, **(spec.get("labels") or {})}),
           "--head-address", head_sock, "--ready-file", ready]
    if ncpu is not None:
        cmd += ["--num-cpus", str(int(ncpu))]
    if ngpu is not None:
        cmd += ["--num-gpus", str(int(ngpu))]
    env = dict(_os.environ)
    pkg = _os.path.dirname(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))))
    env["PYTHONPATH"] = pkg + (_os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    out = open(_os.path.join(session, f"node_{tag}.out"), "ab")
    p = _subprocess.Popen(cmd, env=env, close_fds=True, start_new_session=True, stdout=out,
                          stderr=_subprocess.STDOUT, stdin=_subprocess.DEVNULL)
    t0 = _time.time()
    while not _os.path.exists(_os.path.join(session, ready)):
        if p.poll() is not None or _time.time() - t0 > 60:
            raise RuntimeError(f"{ntype} node failed to start (see {out.name})")
        _time.sleep(0.05)
    return p.pid


def create_or_update_cluster(cluster_config, *, no_restart: bool = False,
                             restart_only: bool = False, no_config_cache: bool = False) -> dict:
    """Bring the cluster up (or bring a running one to ``min_workers`` of every worker
    type). Returns the cluster state: session address, head and worker pids."""
    from ray_amd._private import worker as W

    cfg = bootstrap_config(cluster_config, no_config_cache)
    name = cfg["cluster_name"]
    _fire("up_started", {"cluster_name": name})
    st = _read_state(name)
    if st and _alive(st["head_pid"]) and not restart_only:
        if no_restart:
            return st
    else:
        if st:
            teardown_cluster(cfg)
        _run_cmds(cfg.get("initialization_commands"))
        _run_cmds(cfg.get("setup_commands"))
        _run_cmds(cfg.get("head_setup_commands"))
        head = cfg["available_node_types"][cfg["head_node_type"]]
        res = dict(head.get("resources") or {})
        session = W.new_session_dir()
        proc, _ = W._start_raylet(session, res.pop("CPU", None), res.pop("GPU", None), res,
                                  int(head.get("object_store_memory", 256 << 20)),
                                  {"ray.io/node-type": cfg["head_node_type"]},
                                  detach_output=True)
        st = {"cluster_name": name, "address": session, "head_pid": proc.pid,
              "workers": [], "config": cfg}
        for src, dst in (cfg.get("file_mounts") or {}).items():
            rsync(cfg, source=src, target=dst, down=False)
        _run_cmds(cfg.get("head_start_ray_commands"),
                  env={**_os.environ, "RAY_ADDRESS": session})
        _fire("head_started", {"address": session})
    sock = _os.path.join(st["address"], "sockets", "raylet.sock")
    st["workers"] = [w for w in st["workers"] if _alive(w["pid"])]
    for ntype, spec in cfg["available_node_types"].items():
        if ntype == cfg["head_node_type"]:
            continue
        have = sum(1 for w in st["workers"] if w["type"] == ntype)
        for _ in range(max(0, int(spec.get("min_workers", 0)) - have)):
            _run_cmds(cfg.get("worker_setup_commands"))
            pid = _start_node(st["address"], ntype, spec, sock)
            st["workers"].append({"type": ntype, "pid": pid})
            _fire("worker_started", {"type": ntype, "pid": pid})
    _os.makedirs(_STATE_DIR, exist_ok=True)
    with open(_state_file(name), "w") as f:
        _json.dump(st, f)
    _fire("up_completed", {"cluster_name": name, "address": st["address"]})
    return st


def teardown_cluster(cluster_config, workers_only: bool = False,
                     keep_min_workers: bool = False) -> None:
    """Stop the cluster's node processes (``workers_only``: keep the head)."""
    import signal

    cfg = fillout_defaults(_load(cluster_config))
    name = cfg["cluster_name"]
    st = _read_state(name)
    if not st:
        return
    keep = []
    mins = {t: int(s.get("min_workers", 0)) for t, s in cfg["available_node_types"].items()}
    for w in st["workers"]:
        if keep_min_workers and sum(1 for k in keep if k["type"] == w["type"]) < \
                mins.get(w["type"], 0):
            keep.append(w)
            continue
        if _alive(w["pid"]):
            _os.kill(w["pid"], signal.SIGTERM)
    st["workers"] = keep
    if not workers_only and _alive(st["head_pid"]):
        _os.kill(st["head_pid"], signal.SIGTERM)
        t0 = _time.time()
        while _alive(st["head_pid"]) and _time.time() - t0 < 10:
            _time.sleep(0.05)
        if _alive(st["head_pid"]):
            _os.kill(st["head_pid"], signal.SIGKILL)
    if workers_only:
        with open(_state_file(name), "w") as f:
            _json.dump(st, f)
    else:
        try:
            _os.unlink(_state_file(name))
        except FileNotFoundError:
            pass
    _fire("down_completed", {"cluster_name": name})


def run_on_cluster(cluster_config, *, cmd: str | None = None, run_env: str = "auto",
                   tmux: bool = False, stop: bool = False, no_config_cache: bool = False,
                   port_forward=None, with_output: bool = False):
    """Run ``cmd`` on the head node (here: this machine) with RAY_ADDRESS set to the
    cluster; returns the output with ``with_output``."""
    cfg = fillout_defaults(_load(cluster_config))
    st = _read_state(cfg["cluster_name"])
    if not st:
        raise RuntimeError(f"cluster {cfg['cluster_name']!r} is not running")
    r = _subprocess.run(cmd, shell=True, check=True, capture_output=with_output,
                        text=True, env={**_os.environ, "RAY_ADDRESS": st["address"]})
    if stop:
        teardown_cluster(cfg)
    return r.stdout if with_output else None


def rsync(cluster_config, *, source: str | None, target: str | None, down: bool,
          ip_address: str | None = None, use_internal_ip: bool = False,
          no_config_cache: bool = False, should_bootstrap: bool = True):
    """Copy files to (``down=False``) or from the cluster's nodes. Every node of the
    local provider shares this filesystem, so this is a local copy."""
    src, dst = (source, target)
    if not src or not dst:
        raise ValueError("rsync needs a source and a target")
    src, dst = _os.path.expanduser(src), _os.path.expanduser(dst)
    if _os.path.isdir(src):
        _shutil.copytree(src, dst, dirs_exist_ok=True)
    else:
        _os.makedirs(_os.path.dirname(_os.path.abspath(dst)), exist_ok=True)
        _shutil.copy2(src, dst)


def get_head_node_ip(cluster_config) -> str:
    cfg = fillout_defaults(_load(cluster_config))
    if not _read_state(cfg["cluster_name"]):
        raise RuntimeError(f"cluster {cfg['cluster_name']!r} is not running")
    return "127.0.0.1"


def get_worker_node_ips(cluster_config) -> list:
    cfg = fillout_defaults(_load(cluster_config))
    st = _read_state(cfg["cluster_name"])
    if not st:
        raise RuntimeError(f"cluster {cfg['cluster_name']!r} is not running")
    return ["127.0.0.1" for w in st["workers"] if _alive(w["pid"])]
