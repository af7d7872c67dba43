"""``serve`` CLI (reference: python/ray/serve/scripts.py): start / run / deploy / status /
config / shutdown / build against a running ray_amd cluster.

    python -m ray_amd.serve deploy config.yaml            # declarative, returns at once
    python -m ray_amd.serve run app_module:app k=v ...     # deploy and block (Ctrl-C stops)
    python -m ray_amd.serve status | config | shutdown -y
    python -m ray_amd.serve build app_module:app -o config.yaml

``run``/``deploy`` take either a config file (``*.yaml``/``*.yml``) or an import path; with
an import path, trailing ``key=value`` arguments go to an application builder."""

from __future__ import annotations

import argparse
import os
import sys
import time


def _connect(address):
    import ray_amd as ray

    if not ray.is_initialized():
        ray.init(address=address or "auto", namespace="serve")
    return ray


def _rest(address):
    """The dashboard URL when --address is one (reference: the serve CLI talks to the
    dashboard's /api/serve/applications/ REST API)."""
    return address.rstrip("/") if address and address.startswith("http") else None


def _http(method, url, body=None):
    import requests

    r = requests.request(method, url, json=body, timeout=300)
    if r.status_code >= 400:
        raise SystemExit(f"{method} {url} -> {r.status_code}: {r.text}")
    return r


def _is_config(p: str) -> bool:
    return p.endswith((".yaml", ".yml", ".json")) and os.path.exists(p)


def _config_from(a):
    from ray_amd.serve.schema import ServeDeploySchema, load_config_file

    if _is_config(a.config_or_import_path):
        cfg = load_config_file(a.config_or_import_path)
        if a.arguments:
            raise SystemExit("key=value arguments only apply to an import path")
        return cfg
    args = {}
    for kv in a.arguments or ():
        k, sep, v = kv.partition("=")
        if not sep:
            raise SystemExit(f"argument {kv!r} is not key=value")
        args[k] = v
    wd = a.working_dir or os.getcwd()
    app = {"name": a.name or "default", "route_prefix": a.route_prefix or "/",
           "import_path": a.config_or_import_path, "args": args,
           "runtime_env": {"working_dir": os.path.abspath(wd)}}
    http = {}
    if getattr(a, "port", None):
        http["port"] = a.port
    return ServeDeploySchema(applications=[app], http_options=http)


def _dump(obj):
    import yaml

    print(yaml.safe_dump(obj, sort_keys=False).rstrip())


def cmd_start(a):
    _connect(a.address)
    from ray_amd import serve
    from ray_amd.serve.api import HTTPOptions

    serve.start(http_options=HTTPOptions(host=a.http_host, port=a.http_port,
                                         location={"Disabled": "NoServer",
                                                   "EveryNode": "EveryNode"}.get(
                                             a.proxy_location, "HeadOnly")))
    print(f"Serve started (HTTP {a.http_host}:{a.http_port}).")
    return 0


def cmd_deploy(a):
    url = _rest(a.address)
    if url:
        cfg = _config_from(a)
        _http("PUT", url + "/api/serve/applications/", cfg.model_dump(mode="json"))
        print(f"Sent deploy request for applications: {[x.name for x in cfg.applications]}")
        return 0
    _connect(a.address)
    from ray_amd.serve.schema import deploy_config

    cfg = _config_from(a)
    deploy_config(cfg)
    print(f"Deployed applications: {[x.name for x in cfg.applications]}")
    return 0


def cmd_run(a):
    _connect(a.address)
    from ray_amd import serve
    from ray_amd.serve.schema import deploy_config

    cfg = _config_from(a)
    deploy_config(cfg)
    print(f"Running applications: {[x.name for x in cfg.applications]}", flush=True)
    if a.non_blocking:
        return 0
    try:
        while True:
            time.sleep(1)
    except KeyboardInterrupt:
        print("Shutting down Serve.")
        serve.shutdown()
    return 0


def cmd_status(a):
    url = _rest(a.address)
    if url:
        d = _http("GET", url + "/api/serve/applications/").json()
        _dump({"applications": {n: {k: v for k, v in app.items()
                                    if k not in ("name", "deployed_app_config")}
                                for n, app in d["applications"].items()}})
        return 0
    _connect(a.address)
    from ray_amd import serve

    try:
        st = serve.status()
    except RuntimeError:
        st = {}
    _dump({"applications": st})
    return 0


def cmd_config(a):
    url = _rest(a.address)
    if url:
        d = _http("GET", url + "/api/serve/applications/").json()
        cfg = {"applications": [app["deployed_app_config"] for app in
                                d["applications"].values() if "deployed_app_config" in app]}
    else:
        _connect(a.address)
        from ray_amd.serve.schema import get_deployed_config

        cfg = get_deployed_config()
    if cfg is None:
        print("No configuration was deployed.")
        return 0
    apps = cfg.get("applications", [])
    if a.name:
        apps = [x for x in apps if x.get("name") == a.name]
    for i, app in enumerate(apps):
        if i:
            print("---")
        _dump(app)
    return 0


def cmd_shutdown(a):
    if not a.yes:
        ans = input("This shuts down Serve and deletes every application. Continue? [y/N] ")
        if ans.strip().lower() not in ("y", "yes"):
            return 1
    url = _rest(a.address)
    if url:
        _http("DELETE", url + "/api/serve/applications/")
        print("Serve shut down.")
        return 0
    _connect(a.address)
    from ray_amd import serve

    serve.shutdown()
    print("Serve shut down.")
    return 0


def cmd_build(a):
    from ray_amd.serve.schema import build_config

    wd = os.path.abspath(a.working_dir or os.getcwd())
    if wd not in sys.path:
        sys.path.insert(0, wd)
    out = build_config(a.import_path, name=a.name, route_prefix=a.route_prefix,
                       working_dir=wd)
    import yaml

    text = yaml.safe_dump(out, sort_keys=False)
    if a.output_path:
        with open(a.output_path, "w") as f:
            f.write(text)
    else:
        print(text.rstrip())
    return 0


def build_parser():
    ap = argparse.ArgumentParser(prog="serve", description="ray_amd Serve CLI")
    sub = ap.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("start", help="start Serve (controller + proxy) on the cluster")
    s.add_argument("--address")
    s.add_argument("--http-host", default="127.0.0.1")
    s.add_argument("--http-port", type=int, default=8000)
    s.add_argument("--proxy-location", default="HeadOnly",
                   choices=["HeadOnly", "EveryNode", "Disabled"])
    s.set_defaults(fn=cmd_start)
    for name, fn, hlp in (("deploy", cmd_deploy, "deploy a config file or import path"),
                          ("run", cmd_run, "deploy and block until Ctrl-C")):
        s = sub.add_parser(name, help=hlp)
        s.add_argument("config_or_import_path")
        s.add_argument("arguments", nargs="*")
        s.add_argument("--address")
        s.add_argument("--name", default=None)
        s.add_argument("--route-prefix", default=None)
        s.add_argument("--working-dir", default=None)
        s.add_argument("--port", type=int, default=None)
        if name == "run":
            s.add_argument("--non-blocking", action="store_true")
        s.set_defaults(fn=fn)
    s = sub.add_parser("status", help="application and deployment status (YAML)")
    s.add_argument("--address")
    s.set_defaults(fn=cmd_status)
    s = sub.add_parser("config", help="the last deployed config (YAML)")
    s.add_argument("--address")
    s.add_argument("--name", default=None)
    s.set_defaults(fn=cmd_config)
    s = sub.add_parser("shutdown", help="delete every application and stop Serve")
    s.add_argument("--address")
    s.add_argument("-y", "--yes", action="store_true")
    s.set_defaults(fn=cmd_shutdown)
    s = sub.add_parser("build", help="write a config file for an application")
    s.add_argument("import_path")
    s.add_argument("-o", "--output-path", default=None)
    s.add_argument("--name", default="default")
    s.add_argument("--route-prefix", default="/")
    s.add_argument("--working-dir", default=None)
    s.set_defaults(fn=cmd_build)
    return ap


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    return a.fn(a)


if __name__ == "__main__":
    sys.exit(main())
