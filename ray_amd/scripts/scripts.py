"""``ray_amd`` command line (parity with ``python/ray/scripts/scripts.py``: ``ray start``,
``ray stop``, ``ray status``, ``ray list/get/summary`` (util/state/state_cli.py),
``ray memory``, ``ray timeline``, ``ray microbenchmark``, ``ray metrics``, and
``ray job submit/status/logs/stop/list/delete`` (dashboard/modules/job/cli.py)).

    python -m ray_amd.scripts start --head [--num-cpus N] [--num-gpus N] [--port-dashboard 8265]
    python -m ray_amd.scripts status
    python -m ray_amd.scripts job submit -- python my_script.py
    python -m ray_amd.scripts stop
"""

from __future__ import annotations

import argparse
import json
import os
import signal
import sys
import time


def _session():
    from ray_amd._private.worker import CURRENT_CLUSTER_FILE

    if not os.path.exists(CURRENT_CLUSTER_FILE):
        return None
    with open(CURRENT_CLUSTER_FILE) as f:
        s = f.read().strip()
    return s if os.path.isdir(s) else None


def _connect(address=None):
    import ray_amd as ray

    ray.init(address=address or "auto", namespace="_cli")
    return ray


# ---------------------------------------------------------------------------- start / stop
def _start_worker_node(a):
    """`start --address=<head session>`: join a running cluster as a worker node."""
    import subprocess

    session = _session() if a.address in (None, "auto") else a.address
    if not session or not os.path.isdir(session):
        print("No head node to join: pass --address=<session dir> or start one with "
              "`start --head`.", file=sys.stderr)
        return 1
    from ray_amd._private import worker as W

    osm = int(a.object_store_memory or W._default_object_store_memory() // 4)
    tag = os.urandom(4).hex()
    ready = f"node_{tag}.ready"
    cmd = [sys.executable, "-m", "ray_amd._private.raylet", "--session-dir", session,
           "--store-path", f"/dev/shm/ray_amd_{os.path.basename(session)}_{tag}",
           "--object-store-memory", str(osm), "--resources", a.resources or "{}",
           "--labels", a.labels or "{}", "--head-address",
           os.path.join(session, "sockets", "raylet.sock"), "--ready-file", ready]
    if a.num_cpus is not None:
        cmd += ["--num-cpus", str(a.num_cpus)]
    if a.num_gpus is not None:
        cmd += ["--num-gpus", str(a.num_gpus)]
    env = dict(os.environ)
    pkg = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env["PYTHONPATH"] = pkg + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    out = open(os.path.join(session, f"node_{tag}.out"), "ab")
    proc = subprocess.Popen(cmd, env=env, close_fds=True, start_new_session=True, stdout=out,
                            stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL)
    t0 = time.time()
    while not os.path.exists(os.path.join(session, ready)):
        if proc.poll() is not None or time.time() - t0 > 60:
            print("worker node failed to start", file=sys.stderr)
            return 1
        time.sleep(0.05)
    pf = os.path.join(session, "cluster_pids.json")
    pids = {}
    if os.path.exists(pf):
        with open(pf) as f:
            pids = json.load(f)
    pids.setdefault("nodes", []).append(proc.pid)
    with open(pf, "w") as f:
        json.dump(pids, f)
    print(f"ray_amd worker node started (pid {proc.pid}) and joined {session}")
    return 0


def cmd_start(a):
    from ray_amd._private import worker as W

    if not a.head:
        return _start_worker_node(a)
    if _session() is not None:
        print(f"A ray_amd cluster is already running at {_session()}; run `stop` first.",
              file=sys.stderr)
        return 1
    session = W.new_session_dir()
    osm = int(a.object_store_memory or W._default_object_store_memory())
    resources = json.loads(a.resources) if a.resources else None
    labels = json.loads(a.labels) if a.labels else None
    proc, _addr = W._start_raylet(session, a.num_cpus, a.num_gpus, resources, osm, labels,
                                  detach_output=True)
    pids = {"raylet": proc.pid}
    if getattr(a, "ray_client_server_port", None):
        import subprocess

        env = dict(os.environ)
        pkg = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env["PYTHONPATH"] = pkg + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH")
                                   else "")
        out = open(os.path.join(session, "client_server.out"), "ab")
        cs = subprocess.Popen([sys.executable, "-m", "ray_amd.util.client.server", "--address",
                               session, "--port", str(a.ray_client_server_port)], env=env,
                              stdout=out, stderr=subprocess.STDOUT, stdin=subprocess.DEVNULL,
                              start_new_session=True, close_fds=True)
        pids["client_server"] = cs.pid
    url = None
    if a.include_dashboard:
        from ray_amd.dashboard import start_dashboard

        dproc, url = start_dashboard(session, a.dashboard_host, a.dashboard_port)
        pids["dashboard"] = dproc.pid
    with open(os.path.join(session, "cluster_pids.json"), "w") as f:
        json.dump(pids, f)
    os.makedirs(os.path.dirname(W.CURRENT_CLUSTER_FILE), exist_ok=True)
    with open(W.CURRENT_CLUSTER_FILE, "w") as f:
        f.write(session)
    print("ray_amd runtime started.")
    print(f"  address:   {session}")
    if url:
        print(f"  dashboard: {url}")
    print("  connect with ray_amd.init(address='auto'); stop with "
          "`python -m ray_amd.scripts stop`.")
    if a.block:
        try:
            while proc.poll() is None:
                time.sleep(1)
        except KeyboardInterrupt:
            pass
    return 0


def _pid_alive(pid):
    try:
        os.kill(pid, 0)
        return True
    except ProcessLookupError:
        return False
    except PermissionError:
        return True


def cmd_stop(a):
    from ray_amd._private.worker import CURRENT_CLUSTER_FILE

    session = _session()
    if session is None:
        print("No running ray_amd cluster found.")
        return 0
    pids = {}
    try:
        with open(os.path.join(session, "cluster_pids.json")) as f:
            pids = json.load(f)
    except FileNotFoundError:
        pass
    # dashboard first (it is a driver of the cluster), then the raylet, which reaps workers
    for name in ("client_server", "dashboard", "raylet"):
        pid = pids.get(name)
        if pid and _pid_alive(pid):
            os.kill(pid, signal.SIGKILL if a.force else signal.SIGTERM)
            t0 = time.time()
            while _pid_alive(pid) and time.time() - t0 < a.grace_period:
                time.sleep(0.05)
            if _pid_alive(pid):
                os.kill(pid, signal.SIGKILL)
    for pid in pids.get("nodes", []):  # worker-node agents exit with the head; make sure
        if _pid_alive(pid):
            os.kill(pid, signal.SIGKILL)
    try:
        os.unlink(CURRENT_CLUSTER_FILE)
    except FileNotFoundError:
        pass
    print(f"Stopped ray_amd cluster at {session}.")
    return 0


# ---------------------------------------------------------------------------- status & state
def cmd_status(a):
    ray = _connect(a.address)
    tot = ray.cluster_resources()
    av = ray.available_resources()
    nodes = [n for n in ray.nodes() if n["Alive"]]
    print("======== ray_amd cluster status ========")
    print(f"Nodes: {len(nodes)} alive")
    for n in nodes:
        print(f"  {n['NodeID'][:12]}  {n['NodeManagerHostname']}")
    print("Resources (used / total):")
    for k in sorted(tot):
        used = tot[k] - av.get(k, 0.0)
        unit = ""
        t, u = tot[k], used
        if k in ("memory", "object_store_memory"):
            t, u, unit = t / 2 ** 30, u / 2 ** 30, " GiB"
        print(f"  {u:g}/{t:g}{unit} {k}")
    from ray_amd._private.worker import _check_connected

    try:
        stats = _check_connected().call_raylet("node_stats") or {}
    except Exception:  # noqa: BLE001
        stats = {}
    if stats:
        print("Node telemetry:")
    for nid, s in stats.items():
        print(f"  {nid[:12]}  cpu {s['cpu_percent']:.0f}% of {s['cpu_count']}  mem "
              f"{s['mem_used'] / 2 ** 30:.1f}/{s['mem_total'] / 2 ** 30:.1f} GiB")
        for g in s.get("gpus") or []:
            def f(v, scale=1.0, fmt="{:.0f}"):
                return "n/a" if v is None else fmt.format(v / scale)

            print(f"    GPU{g['index']} {g['name']}: util {f(g['utilization_percent'])}%  "
                  f"HBM {f(g['memory_used'], 2 ** 30, '{:.1f}')}/"
                  f"{f(g['memory_total'], 2 ** 30, '{:.1f}')} GiB  power "
                  f"{f(g['power_w'])} W  temp {f(g['temperature_c'])} C")
    return 0


def _print_rows(rows, fmt):
    rows = [dict(r) for r in rows]
    if fmt == "json":
        print(json.dumps(rows, indent=2, default=str))
        return
    if fmt == "yaml":
        import yaml

        print(yaml.safe_dump(rows, sort_keys=False, default_flow_style=False))
        return
    if not rows:
        print("(no entries)")
        return
    cols = list(rows[0].keys())[:8]
    try:
        from tabulate import tabulate

        print(tabulate([[str(r.get(c))[:40] for c in cols] for r in rows], headers=cols))
    except ImportError:
        for r in rows:
            print({c: r.get(c) for c in cols})


def _filters(specs):
    out = []
    for s in specs or ():
        for pred in ("!=", "="):
            if pred in s:
                k, v = s.split(pred, 1)
                out.append((k.strip(), pred, v.strip()))
                break
        else:
            raise SystemExit(f"bad filter {s!r}; use key=value or key!=value")
    return out


def cmd_list(a):
    _connect(a.address)
    from ray_amd.util.state import StateApiClient

    rows = StateApiClient().list(a.resource, filters=_filters(a.filter), limit=a.limit)
    _print_rows(rows, a.format)
    return 0


def cmd_get(a):
    _connect(a.address)
    from ray_amd.util import state

    fn = {"actors": state.get_actor, "tasks": state.get_task, "nodes": state.get_node,
          "workers": state.get_worker, "placement-groups": state.get_placement_group,
          "placement_groups": state.get_placement_group, "jobs": state.get_job,
          "objects": state.get_objects}[a.resource]
    r = fn(a.id)
    if r is None:
        print(f"{a.resource[:-1]} {a.id} not found", file=sys.stderr)
        return 1
    print(json.dumps(r if isinstance(r, (dict, list)) else dict(r), indent=2, default=str))
    return 0


def cmd_summary(a):
    _connect(a.address)
    from ray_amd.util import state

    fn = {"tasks": state.summarize_tasks, "actors": state.summarize_actors,
          "objects": state.summarize_objects}[a.resource]
    print(json.dumps(fn(), indent=2, default=str))
    return 0


def cmd_memory(a):
    _connect(a.address)
    from ray_amd.util import state

    objs = state.list_objects(limit=None)
    total = sum(o.object_size or 0 for o in objs)
    print(f"{len(objs)} objects, {total / 2 ** 20:.1f} MiB")
    _print_rows(objs[: a.limit], "table")
    return 0


def cmd_debug(a):
    """List live remote-pdb breakpoints (util.rpdb) and attach the terminal to one."""
    import time

    _connect(a.address)
    from ray_amd.util import rpdb

    deadline = time.time() + a.wait
    bps = rpdb.list_breakpoints()
    while not bps and time.time() < deadline:
        time.sleep(0.5)
        bps = rpdb.list_breakpoints()
    if not bps:
        print("No active breakpoints.")
        return 0
    for i, b in enumerate(bps):
        print(f"{i}: pid={b['pid']} {b['host']}:{b['port']} task={b.get('task_id')} "
              f"actor={b.get('actor_id')}")
    idx = a.index
    if idx is None:
        if len(bps) == 1 or not sys.stdin.isatty():
            idx = 0
        else:
            idx = int(input("Enter breakpoint index: "))
    b = bps[idx]
    rpdb.connect_pdb_client(b["host"], b["port"])
    return 0


def cmd_logs(a):
    """`logs` lists session log files; `logs <file>` / `logs --pid N` prints one."""
    _connect(a.address)
    from ray_amd.util import state

    if a.filename is None and a.pid is None and a.actor_id is None:
        for cat, files in state.list_logs(glob_filter=a.glob).items():
            if files:
                print(f"{cat}:")
                for f in files:
                    print(f"  {f}")
        return 0
    for ln in state.get_log(filename=a.filename, pid=a.pid, actor_id=a.actor_id, tail=a.tail,
                            follow=a.follow, suffix="err" if a.err else "out"):
        print(ln)
    return 0


def cmd_timeline(a):
    ray = _connect(a.address)
    out = a.output or f"/tmp/ray_amd-timeline-{time.strftime('%Y-%m-%d_%H-%M-%S')}.json"
    ray.timeline(filename=out)
    print(f"Trace file written to {out} (open in chrome://tracing or Perfetto).")
    return 0


def cmd_metrics(a):
    _connect(a.address)
    from ray_amd.util.metrics import prometheus_text

    sys.stdout.write(prometheus_text())
    return 0


def cmd_up(a):
    from ray_amd.autoscaler import sdk

    st = sdk.create_or_update_cluster(a.cluster_config, no_restart=a.no_restart,
                                      restart_only=a.restart_only)
    print(f"Cluster {st['cluster_name']} is up: address {st['address']}, "
          f"{len(st['workers'])} worker node(s). Connect with "
          f"ray_amd.init(address='{st['address']}').")
    return 0


def cmd_down(a):
    from ray_amd.autoscaler import sdk

    sdk.teardown_cluster(a.cluster_config, workers_only=a.workers_only,
                         keep_min_workers=a.keep_min_workers)
    print("Cluster torn down." if not a.workers_only else "Worker nodes torn down.")
    return 0


def cmd_exec(a):
    from ray_amd.autoscaler import sdk

    sdk.run_on_cluster(a.cluster_config, cmd=a.cmd)
    return 0


def cmd_rsync(a):
    from ray_amd.autoscaler import sdk

    sdk.rsync(a.cluster_config, source=a.source, target=a.target, down=a.down)
    return 0


def cmd_ips(a):
    from ray_amd.autoscaler import sdk

    if a.which == "get-head-ip":
        print(sdk.get_head_node_ip(a.cluster_config))
    else:
        print("\n".join(sdk.get_worker_node_ips(a.cluster_config)))
    return 0


def cmd_microbenchmark(a):
    from ray_amd._private import ray_perf

    ray_perf.main(quick=a.quick)
    return 0


# ---------------------------------------------------------------------------- jobs
def _client(a):
    from ray_amd.job_submission import JobSubmissionClient

    return JobSubmissionClient(a.address)


def cmd_job_submit(a):
    from ray_amd.job_submission import JobStatus

    c = _client(a)
    ep = list(a.entrypoint)
    if ep and ep[0] == "--":
        ep = ep[1:]
    renv = json.loads(a.runtime_env_json) if a.runtime_env_json else {}
    if a.working_dir:
        renv["working_dir"] = a.working_dir
    jid = c.submit_job(entrypoint=" ".join(ep), submission_id=a.submission_id, runtime_env=renv,
                       metadata=json.loads(a.metadata_json) if a.metadata_json else None,
                       entrypoint_num_cpus=a.entrypoint_num_cpus,
                       entrypoint_num_gpus=a.entrypoint_num_gpus)
    print(f"Job '{jid}' submitted successfully")
    if a.no_wait:
        return 0
    import asyncio

    async def follow():
        async for chunk in c.tail_job_logs(jid):
            sys.stdout.write(chunk)
            sys.stdout.flush()

    asyncio.run(follow())
    st = c.wait_until_status(jid, {JobStatus.SUCCEEDED, JobStatus.FAILED, JobStatus.STOPPED},
                             timeout_s=3600)
    print(f"Job '{jid}' {'succeeded' if st == JobStatus.SUCCEEDED else str(st).lower()}")
    return 0 if st == JobStatus.SUCCEEDED else 1


def cmd_job_status(a):
    info = _client(a).get_job_info(a.job_id)
    print(f"Status for job '{a.job_id}': {info.status}")
    if info.message:
        print(f"Status message: {info.message}")
    return 0


def cmd_job_logs(a):
    c = _client(a)
    if a.follow:
        import asyncio

        async def follow():
            async for chunk in c.tail_job_logs(a.job_id):
                sys.stdout.write(chunk)

        asyncio.run(follow())
    else:
        sys.stdout.write(c.get_job_logs(a.job_id))
    return 0


def cmd_job_stop(a):
    ok = _client(a).stop_job(a.job_id)
    print(f"Job '{a.job_id}' {'stopped' if ok else 'was not running'}")
    return 0


def cmd_job_list(a):
    jobs = _client(a).list_jobs()
    _print_rows([{"submission_id": j.submission_id, "status": str(j.status),
                  "entrypoint": j.entrypoint, "start_time": j.start_time} for j in jobs], "table")
    return 0


def cmd_job_delete(a):
    _client(a).delete_job(a.job_id)
    print(f"Job '{a.job_id}' deleted successfully")
    return 0


# ---------------------------------------------------------------------------- parser
def build_parser():
    p = argparse.ArgumentParser(prog="ray_amd")
    sub = p.add_subparsers(dest="cmd", required=True)

    s = sub.add_parser("start", help="start a head node")
    s.add_argument("--head", action="store_true")
    s.add_argument("--address", help="join this cluster (session dir or 'auto') as a worker node")
    s.add_argument("--num-cpus", type=int)
    s.add_argument("--num-gpus", type=int)
    s.add_argument("--resources")
    s.add_argument("--labels")
    s.add_argument("--object-store-memory", type=int)
    s.add_argument("--include-dashboard", type=lambda v: v.lower() in ("1", "true", "yes"),
                   default=True)
    s.add_argument("--dashboard-host", default="127.0.0.1")
    s.add_argument("--dashboard-port", type=int, default=8265)
    s.add_argument("--block", action="store_true")
    s.add_argument("--ray-client-server-port", type=int, default=None,
                   help="also serve Ray Client connections (ray://127.0.0.1:<port>)")
    s.set_defaults(fn=cmd_start)

    s = sub.add_parser("stop", help="stop the running cluster")
    s.add_argument("-f", "--force", action="store_true")
    s.add_argument("-g", "--grace-period", type=float, default=10.0)
    s.set_defaults(fn=cmd_stop)

    for name, fn in (("status", cmd_status), ("timeline", cmd_timeline),
                     ("metrics", cmd_metrics)):
        s = sub.add_parser(name)
        s.add_argument("--address")
        if name == "timeline":
            s.add_argument("--output")
        s.set_defaults(fn=fn)

    s = sub.add_parser("list", help="list cluster state (actors, tasks, objects, ...)")
    s.add_argument("resource", choices=["actors", "tasks", "objects", "nodes", "workers", "jobs",
                                        "placement-groups", "placement_groups", "runtime-envs",
                                        "runtime_envs"])
    s.add_argument("--filter", action="append")
    s.add_argument("--limit", type=int, default=100)
    s.add_argument("--format", choices=["table", "json", "yaml"], default="table")
    s.add_argument("--address")
    s.set_defaults(fn=lambda a: cmd_list(_norm(a)))

    s = sub.add_parser("get")
    s.add_argument("resource")
    s.add_argument("id")
    s.add_argument("--address")
    s.set_defaults(fn=cmd_get)

    s = sub.add_parser("summary")
    s.add_argument("resource", choices=["tasks", "actors", "objects"])
    s.add_argument("--address")
    s.set_defaults(fn=cmd_summary)

    s = sub.add_parser("memory")
    s.add_argument("--address")
    s.add_argument("--limit", type=int, default=50)
    s.set_defaults(fn=cmd_memory)

    s = sub.add_parser("logs", help="list / print worker log files")
    s.add_argument("filename", nargs="?")
    s.add_argument("--address")
    s.add_argument("--pid", type=int)
    s.add_argument("--actor-id")
    s.add_argument("--glob")
    s.add_argument("--tail", type=int, default=-1)
    s.add_argument("--err", action="store_true")
    s.add_argument("-f", "--follow", action="store_true")
    s.set_defaults(fn=cmd_logs)

    s = sub.add_parser("debug", help="attach to a remote pdb breakpoint (util.pdb.set_trace)")
    s.add_argument("--address")
    s.add_argument("--index", type=int)
    s.add_argument("--wait", type=float, default=0.0, help="seconds to wait for a breakpoint")
    s.set_defaults(fn=cmd_debug)

    # cluster launcher (reference: `ray up/down/exec/rsync-up/rsync-down/get-head-ip`)
    s = sub.add_parser("up", help="start or update a cluster from a cluster YAML")
    s.add_argument("cluster_config")
    s.add_argument("--no-restart", action="store_true")
    s.add_argument("--restart-only", action="store_true")
    s.add_argument("-y", "--yes", action="store_true")
    s.set_defaults(fn=cmd_up)
    s = sub.add_parser("down", help="tear a cluster down")
    s.add_argument("cluster_config")
    s.add_argument("--workers-only", action="store_true")
    s.add_argument("--keep-min-workers", action="store_true")
    s.add_argument("-y", "--yes", action="store_true")
    s.set_defaults(fn=cmd_down)
    s = sub.add_parser("exec", help="run a command on the cluster's head node")
    s.add_argument("cluster_config")
    s.add_argument("cmd")
    s.set_defaults(fn=cmd_exec)
    for name, down in (("rsync-up", False), ("rsync-down", True)):
        s = sub.add_parser(name)
        s.add_argument("cluster_config")
        s.add_argument("source")
        s.add_argument("target")
        s.set_defaults(fn=cmd_rsync, down=down)
    for name in ("get-head-ip", "get-worker-ips"):
        s = sub.add_parser(name)
        s.add_argument("cluster_config")
        s.set_defaults(fn=cmd_ips, which=name)

    s = sub.add_parser("microbenchmark")
    s.add_argument("--quick", action="store_true")
    s.set_defaults(fn=cmd_microbenchmark)

    j = sub.add_parser("job", help="job submission").add_subparsers(dest="jobcmd", required=True)
    s = j.add_parser("submit")
    s.add_argument("--address")
    s.add_argument("--submission-id")
    s.add_argument("--runtime-env-json")
    s.add_argument("--metadata-json")
    s.add_argument("--working-dir")
    s.add_argument("--entrypoint-num-cpus", type=float)
    s.add_argument("--entrypoint-num-gpus", type=float)
    s.add_argument("--no-wait", action="store_true")
    s.add_argument("entrypoint", nargs=argparse.REMAINDER)
    s.set_defaults(fn=cmd_job_submit)
    for name, fn in (("status", cmd_job_status), ("stop", cmd_job_stop),
                     ("delete", cmd_job_delete)):
        s = j.add_parser(name)
        s.add_argument("job_id")
        s.add_argument("--address")
        s.set_defaults(fn=fn)
    s = j.add_parser("logs")
    s.add_argument("job_id")
    s.add_argument("--address")
    s.add_argument("-f", "--follow", action="store_true")
    s.set_defaults(fn=cmd_job_logs)
    s = j.add_parser("list")
    s.add_argument("--address")
    s.set_defaults(fn=cmd_job_list)
    return p


def _norm(a):
    a.resource = a.resource.replace("-", "_")
    return a


def main(argv=None) -> int:
    args = build_parser().parse_args(argv)
    return int(args.fn(args) or 0)


if __name__ == "__main__":
    sys.exit(main())
