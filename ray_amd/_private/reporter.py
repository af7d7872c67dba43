"""Per-node telemetry reporter (reference: python/ray/dashboard/modules/reporter/
reporter_agent.py:277 (GPU stats), :425 (node stats / metric records)).

A ``NodeReporter`` thread runs in every node process (the head raylet and each node agent)
and samples, every ``RAY_AMD_REPORTER_INTERVAL_S`` seconds (default 2):

* host: CPU utilisation, core count, load average, memory total/used/available, the
  session disk, network bytes sent/received;
* per MI355X (any AMD GPU): utilisation (GFX activity), HBM used/total, socket power and
  hotspot/edge temperature — through ``amdsmi`` when the driver answers, else the amdgpu
  sysfs files (``gpu_busy_percent``, ``mem_info_vram_used/total``, hwmon ``power1_average``
  / ``temp*_input``).

``metric_records`` turns a sample into the raylet's gauge records (``ray_node_*`` and
``ray_node_gpus_*`` series, labelled by NodeId and GpuIndex), which the Prometheus
``/metrics`` endpoint, ``util.metrics.prometheus_text`` and ``ray_amd status`` render; the
raw sample is attached to ``/api/v0/nodes`` rows."""

from __future__ import annotations

import glob
import os
import threading
import time

INTERVAL_S = float(os.environ.get("RAY_AMD_REPORTER_INTERVAL_S", "2.0"))


class _AmdSmi:
    """GPU stats through amdsmi (ROCm SMI library); None-returning when unavailable."""

    def __init__(self):
        self.ok = False
        self.handles = []
        try:
            import amdsmi

            amdsmi.amdsmi_init(amdsmi.AmdSmiInitFlags.INIT_AMD_GPUS)
            self.mod = amdsmi
            self.handles = list(amdsmi.amdsmi_get_processor_handles())
            self.ok = bool(self.handles)
        except Exception:  # noqa: BLE001  (no driver here / no GPU)
            self.ok = False

    def sample(self):
        m = self.mod
        out = []
        for i, h in enumerate(self.handles):
            g = {"index": i, "name": "AMD GPU", "utilization_percent": None,
                 "memory_used": None, "memory_total": None, "power_w": None,
                 "temperature_c": None, "source": "amdsmi"}
            try:
                g["name"] = m.amdsmi_get_gpu_asic_info(h).get("market_name") or g["name"]
            except Exception:  # noqa: BLE001
                pass
            try:
                act = m.amdsmi_get_gpu_activity(h)
                v = act.get("gfx_activity")
                g["utilization_percent"] = float(v) if isinstance(v, (int, float)) else None
            except Exception:  # noqa: BLE001
                pass
            try:
                vu = m.amdsmi_get_gpu_vram_usage(h)  # MB
                g["memory_used"] = float(vu["vram_used"]) * 2 ** 20
                g["memory_total"] = float(vu["vram_total"]) * 2 ** 20
            except Exception:  # noqa: BLE001
                pass
            try:
                p = m.amdsmi_get_power_info(h)
                for k in ("current_socket_power", "socket_power", "average_socket_power"):
                    v = p.get(k)
                    if isinstance(v, (int, float)) and v not in (0xFFFF, 0xFFFFFFFF):
                        g["power_w"] = float(v)
                        break
            except Exception:  # noqa: BLE001
                pass
            for kind in ("HOTSPOT", "EDGE"):
                try:
                    t = m.amdsmi_get_temp_metric(h, getattr(m.AmdSmiTemperatureType, kind),
                                                 m.AmdSmiTemperatureMetric.CURRENT)
                    if isinstance(t, (int, float)) and 0 < t < 500:
                        g["temperature_c"] = float(t)
                        break
                except Exception:  # noqa: BLE001
                    continue
            out.append(g)
        return out


def _read(path, conv=float):
    try:
        with open(path) as f:
            return conv(f.read().strip())
    except (OSError, ValueError):
        return None


class _Sysfs:
    """GPU stats from the amdgpu driver's sysfs files."""

    def __init__(self, root="/sys/class/drm"):
        self.cards = []
        for d in sorted(glob.glob(os.path.join(root, "card[0-9]*"))):
            dev = os.path.join(d, "device")
            if os.path.basename(d).count("-"):
                continue  # connectors (card0-DP-1)
            if _read(os.path.join(dev, "vendor"), lambda s: int(s, 16)) != 0x1002:
                continue
            if not os.path.exists(os.path.join(dev, "mem_info_vram_total")):
                continue
            self.cards.append(dev)
        self.ok = bool(self.cards)

    def sample(self):
        out = []
        for i, dev in enumerate(self.cards):
            hw = sorted(glob.glob(os.path.join(dev, "hwmon", "hwmon*")))
            power = temp = None
            if hw:
                pw = _read(os.path.join(hw[0], "power1_average")) or \
                    _read(os.path.join(hw[0], "power1_input"))
                power = pw / 1e6 if pw is not None else None
                for t in ("temp2_input", "temp1_input"):  # junction/hotspot, then edge
                    v = _read(os.path.join(hw[0], t))
                    if v is not None:
                        temp = v / 1e3
                        break
            out.append({"index": i, "name": "AMD GPU",
                        "utilization_percent": _read(os.path.join(dev, "gpu_busy_percent")),
                        "memory_used": _read(os.path.join(dev, "mem_info_vram_used")),
                        "memory_total": _read(os.path.join(dev, "mem_info_vram_total")),
                        "power_w": power, "temperature_c": temp, "source": "sysfs"})
        return out


class NodeReporter:
    def __init__(self, node_id_hex: str, session_dir: str | None = None,
                 interval_s: float = INTERVAL_S, sysfs_root: str = "/sys/class/drm"):
        self.node_id = node_id_hex
        self.session_dir = session_dir or "/tmp"
        self.interval_s = interval_s
        self._gpu = None
        self._sysfs_root = sysfs_root
        self._latest = None
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._thread = None

    def _gpu_backend(self):
        if self._gpu is None:
            b = _AmdSmi()
            if not b.ok:
                b = _Sysfs(self._sysfs_root)
            self._gpu = b
        return self._gpu

    def sample(self) -> dict:
        import psutil

        vm = psutil.virtual_memory()
        try:
            du = psutil.disk_usage(self.session_dir)
            disk = {"total": float(du.total), "used": float(du.used)}
        except OSError:
            disk = None
        try:
            net = psutil.net_io_counters()
            net = {"sent": float(net.bytes_sent), "recv": float(net.bytes_recv)}
        except Exception:  # noqa: BLE001
            net = None
        g = self._gpu_backend()
        try:
            gpus = g.sample() if g.ok else []
        except Exception:  # noqa: BLE001
            gpus = []
        return {"ts": time.time(), "node_id": self.node_id,
                "cpu_percent": float(psutil.cpu_percent(interval=None)),
                "cpu_count": psutil.cpu_count(),
                "load_avg": list(os.getloadavg()),
                "mem_total": float(vm.total), "mem_used": float(vm.total - vm.available),
                "mem_available": float(vm.available), "disk": disk, "net": net,
                "gpus": gpus}

    def latest(self) -> dict | None:
        with self._lock:
            return self._latest

    def _run(self):
        while not self._stop.is_set():
            try:
                s = self.sample()
                with self._lock:
                    self._latest = s
            except Exception:  # noqa: BLE001
                pass
            self._stop.wait(self.interval_s)

    def start(self):
        if self._thread is None:
            self._thread = threading.Thread(target=self._run, daemon=True,
                                            name="node-reporter")
            self._thread.start()
        return self

    def stop(self):
        self._stop.set()


_GAUGES = (
    ("ray_node_cpu_utilization", "Node CPU utilisation (percent)", "cpu_percent"),
    ("ray_node_cpu_count", "Node CPU cores", "cpu_count"),
    ("ray_node_mem_total", "Node memory total (bytes)", "mem_total"),
    ("ray_node_mem_used", "Node memory used (bytes)", "mem_used"),
    ("ray_node_mem_available", "Node memory available (bytes)", "mem_available"),
)
_GPU_GAUGES = (
    ("ray_node_gpus_utilization", "GPU utilisation (percent, GFX activity)",
     "utilization_percent"),
    ("ray_node_gram_used", "GPU HBM used (bytes)", "memory_used"),
    ("ray_node_gram_available", "GPU HBM free (bytes)", None),
    ("ray_node_gram_total", "GPU HBM total (bytes)", "memory_total"),
    ("ray_node_gpu_power_watts", "GPU socket power (W)", "power_w"),
    ("ray_node_gpu_temperature_celsius", "GPU temperature (C)", "temperature_c"),
)
METRIC_NAMES = tuple(n for n, _, _ in _GAUGES) + ("ray_node_load_avg_1m",
                                                   "ray_node_disk_usage",
                                                   "ray_node_network_sent",
                                                   "ray_node_network_received") + \
    tuple(n for n, _, _ in _GPU_GAUGES)


def metric_records(samples) -> list:
    """Gauge records (the raylet's ``get_metrics`` format) for node samples."""
    recs = {n: {"kind": "gauge", "name": n, "description": d, "series": {}}
            for n, d in [(g[0], g[1]) for g in _GAUGES + _GPU_GAUGES] +
            [("ray_node_load_avg_1m", "Node 1-minute load average"),
             ("ray_node_disk_usage", "Session disk used (bytes)"),
             ("ray_node_network_sent", "Network bytes sent"),
             ("ray_node_network_received", "Network bytes received")]}
    for s in samples:
        if not s:
            continue
        node = (("NodeId", s["node_id"]),)
        for name, _, key in _GAUGES:
            if s.get(key) is not None:
                recs[name]["series"][node] = float(s[key])
        recs["ray_node_load_avg_1m"]["series"][node] = float(s["load_avg"][0])
        if s.get("disk"):
            recs["ray_node_disk_usage"]["series"][node] = s["disk"]["used"]
        if s.get("net"):
            recs["ray_node_network_sent"]["series"][node] = s["net"]["sent"]
            recs["ray_node_network_received"]["series"][node] = s["net"]["recv"]
        for g in s.get("gpus") or []:
            lab = node + (("GpuIndex", str(g["index"])), ("GpuDeviceName", g["name"]))
            for name, _, key in _GPU_GAUGES:
                if key is None:
                    if g.get("memory_total") is not None and g.get("memory_used") is not None:
                        recs[name]["series"][lab] = g["memory_total"] - g["memory_used"]
                elif g.get(key) is not None:
                    recs[name]["series"][lab] = float(g[key])
    return list(recs.values())
