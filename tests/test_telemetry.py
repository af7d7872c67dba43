"""Node / MI355X telemetry (reference: dashboard/modules/reporter/reporter_agent.py:277,425):
metric names in the Prometheus text, node stats in the state API, the sysfs GPU backend on
a synthetic amdgpu tree, agent -> head reporting on a two-node cluster, and (GPU) HBM-used
rising after a 1 GiB allocation."""
import os
import time

import pytest

import ray_amd as ray
from ray_amd._private import reporter as R


def test_node_metrics_exported():
    ray.init(num_cpus=2)
    try:
        from ray_amd.util.metrics import prometheus_text
        from ray_amd.util.state import list_nodes

        text = prometheus_text()
        for name in ("ray_node_cpu_utilization", "ray_node_mem_used", "ray_node_mem_total",
                     "ray_node_load_avg_1m"):
            assert f"{name}{{" in text, name
        for name in ("ray_node_gpus_utilization", "ray_node_gram_used",
                     "ray_node_gpu_power_watts", "ray_node_gpu_temperature_celsius"):
            assert f"# TYPE {name} gauge" in text or f"# HELP {name}" in text, name
        rows = list_nodes()
        st = rows[0]["node_stats"]
        assert st["cpu_count"] >= 1 and st["mem_total"] > st["mem_used"] > 0
    finally:
        ray.shutdown()


def _fake_card(root, idx, used, total, busy, power_uw, temp_mc):
    dev = root / f"card{idx}" / "device"
    (dev / "hwmon" / "hwmon3").mkdir(parents=True)
    (dev / "vendor").write_text("0x1002\n")
    (dev / "mem_info_vram_used").write_text(f"{used}\n")
    (dev / "mem_info_vram_total").write_text(f"{total}\n")
    (dev / "gpu_busy_percent").write_text(f"{busy}\n")
    (dev / "hwmon" / "hwmon3" / "power1_average").write_text(f"{power_uw}\n")
    (dev / "hwmon" / "hwmon3" / "temp2_input").write_text(f"{temp_mc}\n")
    (root / f"card{idx}-DP-1").mkdir()  # a connector: ignored


def test_sysfs_backend_and_records(tmp_path):
    _fake_card(tmp_path, 0, 5 * 2 ** 30, 288 * 2 ** 30, 97, 1_250_000_000, 71_000)
    _fake_card(tmp_path, 1, 2 ** 30, 288 * 2 ** 30, 3, 240_000_000, 40_000)
    b = R._Sysfs(str(tmp_path))
    assert b.ok and len(b.cards) == 2
    g0, g1 = b.sample()
    assert g0["memory_used"] == 5 * 2 ** 30 and g0["memory_total"] == 288 * 2 ** 30
    assert g0["utilization_percent"] == 97 and g0["power_w"] == pytest.approx(1250.0)
    assert g0["temperature_c"] == pytest.approx(71.0) and g1["utilization_percent"] == 3
    rep = R.NodeReporter("ab" * 16, str(tmp_path), sysfs_root=str(tmp_path))
    rep._gpu = b
    s = rep.sample()
    recs = {r["name"]: r for r in R.metric_records([s])}
    used = recs["ray_node_gram_used"]["series"]
    key = (("NodeId", "ab" * 16), ("GpuIndex", "0"), ("GpuDeviceName", "AMD GPU"))
    assert used[key] == 5 * 2 ** 30
    assert recs["ray_node_gram_available"]["series"][key] == 283 * 2 ** 30
    assert set(R.METRIC_NAMES) <= set(recs)


def test_agent_reports_to_head():
    from ray_amd.cluster_utils import Cluster

    c = Cluster(initialize_head=True, head_node_args={"num_cpus": 1})
    n1 = c.add_node(num_cpus=1)
    ray.init(address=c.address)
    try:
        from ray_amd._private.worker import _check_connected

        deadline = time.time() + 20
        stats = {}
        while time.time() < deadline:
            stats = _check_connected().call_raylet("node_stats")
            if len(stats) == 2:
                break
            time.sleep(0.2)
        assert len(stats) == 2
        assert all(s["mem_total"] > 0 for s in stats.values())
    finally:
        ray.shutdown()
        c.shutdown()


@pytest.mark.gpu
def test_hbm_used_rises_after_1gib_allocation():
    import torch

    rep = R.NodeReporter("gpu-test", "/tmp")
    b = rep._gpu_backend()
    assert b.ok, "no GPU telemetry backend (amdsmi / amdgpu sysfs) on a GPU box"
    dev = torch.cuda.current_device()
    before = rep.sample()["gpus"]
    x = torch.empty(2 ** 30, dtype=torch.uint8, device="cuda")
    x.fill_(1)
    torch.cuda.synchronize()
    after = rep.sample()["gpus"]
    # the box exposes one card; compare the most-grown card in case indices differ
    grow = max((a["memory_used"] or 0) - (b0["memory_used"] or 0)
               for a, b0 in zip(after, before))
    assert grow >= 0.9 * 2 ** 30, (before, after, dev)
    assert all(g["memory_total"] and g["memory_total"] > 100 * 2 ** 30 for g in after)
    del x
