"""Cluster launcher on the local provider (reference: python/ray/autoscaler/sdk/sdk.py
create_or_update_cluster / teardown_cluster / run_on_cluster / rsync / get_*_ip, and the
`ray up/down/exec/rsync-up/get-head-ip` CLI): every node of the cluster YAML is a process on
this machine."""
import os
import subprocess
import sys

import pytest
import yaml

import ray_amd as ray


@pytest.fixture
def cfg_path(tmp_path, monkeypatch):
    monkeypatch.setenv("RAY_AMD_CLUSTER_STATE_DIR", str(tmp_path / "state"))
    import importlib

    from ray_amd.autoscaler import sdk

    importlib.reload(sdk)
    cfg = {"cluster_name": "t6", "provider": {"type": "local"},
           "head_node_type": "head",
           "available_node_types": {
               "head": {"resources": {"CPU": 1}},
               "cpu_worker": {"resources": {"CPU": 2, "pool": 2}, "min_workers": 2,
                              "max_workers": 3}},
           "setup_commands": [f"touch {tmp_path}/setup_ran"]}
    p = tmp_path / "cluster.yaml"
    p.write_text(yaml.safe_dump(cfg))
    yield str(p), sdk, tmp_path
    sdk.teardown_cluster(str(p))


def test_up_exec_rsync_down(cfg_path):
    path, sdk, tmp = cfg_path
    events = []
    sdk.register_callback_handler("worker_started", lambda d: events.append(d["type"]))
    st = sdk.create_or_update_cluster(path)
    assert os.path.exists(tmp / "setup_ran")
    assert events == ["cpu_worker", "cpu_worker"]
    assert sdk.get_head_node_ip(path) == "127.0.0.1"
    assert len(sdk.get_worker_node_ips(path)) == 2
    ray.init(address=st["address"])
    try:
        @ray.remote(resources={"pool": 1})
        def where():
            return ray.get_runtime_context().get_node_id()

        nodes = {n["NodeID"] for n in ray.nodes() if n["Alive"]}
        assert len(nodes) == 3
        assert ray.get(where.remote()) in nodes
    finally:
        ray.shutdown()
    out = sdk.run_on_cluster(path, cmd="echo $RAY_ADDRESS", with_output=True)
    assert out.strip() == st["address"]
    (tmp / "src.txt").write_text("hello")
    sdk.rsync(path, source=str(tmp / "src.txt"), target=str(tmp / "dst" / "x.txt"), down=False)
    assert (tmp / "dst" / "x.txt").read_text() == "hello"
    # idempotent: a second `up` with no_restart keeps the running cluster
    st2 = sdk.create_or_update_cluster(path, no_restart=True)
    assert st2["address"] == st["address"]
    sdk.teardown_cluster(path, workers_only=True)
    assert sdk.get_worker_node_ips(path) == []
    sdk.teardown_cluster(path)
    with pytest.raises(RuntimeError):
        sdk.get_head_node_ip(path)


def test_cli_up_down(cfg_path):
    path, sdk, tmp = cfg_path
    env = {**os.environ, "RAY_AMD_CLUSTER_STATE_DIR": str(tmp / "state")}
    r = subprocess.run([sys.executable, "-m", "ray_amd.scripts", "up", path, "-y"],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "is up" in r.stdout
    r = subprocess.run([sys.executable, "-m", "ray_amd.scripts", "get-worker-ips", path],
                       capture_output=True, text=True, env=env, timeout=60)
    assert r.stdout.split() == ["127.0.0.1", "127.0.0.1"]
    r = subprocess.run([sys.executable, "-m", "ray_amd.scripts", "down", path, "-y"],
                       capture_output=True, text=True, env=env, timeout=60)
    assert r.returncode == 0, r.stderr


def test_cloud_provider_refused():
    from ray_amd.autoscaler import sdk

    with pytest.raises(ValueError, match="local"):
        sdk.bootstrap_config({"provider": {"type": "aws"}})
    assert sdk.fillout_defaults({})["provider"]["type"] == "local"
