"""Accelerator type detection and scheduling (modelled on python/ray/tests/accelerators/
test_amd_gpu.py)."""

import ray_amd as ray


def test_accelerator_type_detection(tmp_path):
    from ray_amd.util import accelerators as acc

    n = tmp_path / "nodes"
    (n / "0").mkdir(parents=True)
    (n / "0" / "properties").write_text("cpu_cores_count 64\nsimd_count 0\n")
    (n / "1").mkdir()
    (n / "1" / "properties").write_text("simd_count 1024\ngfx_target_version 90500\n"
                                        "device_id 30115\n")  # 0x75a3
    assert acc.detect_accelerator_type(str(n)) == acc.AMD_INSTINCT_MI355x
    (n / "1" / "properties").write_text("simd_count 1024\ngfx_target_version 90500\n"
                                        "device_id 1\n")
    assert acc.detect_accelerator_type(str(n)) == acc.AMD_INSTINCT_MI355x
    (n / "1" / "properties").write_text("simd_count 1024\ngfx_target_version 120001\n")
    assert acc.detect_accelerator_type(str(n)) == "AMD-Instinct-gfx1201"
    assert acc.detect_accelerator_type(str(tmp_path / "none")) is None


def test_accelerator_type_scheduling(monkeypatch):
    from ray_amd.util.accelerators import AMD_INSTINCT_MI355x

    monkeypatch.setenv("RAY_AMD_ACCELERATOR_TYPE", AMD_INSTINCT_MI355x)
    ray.init(num_cpus=2, num_gpus=1)
    try:
        assert ray.cluster_resources().get(f"accelerator_type:{AMD_INSTINCT_MI355x}") == 1.0

        @ray.remote(accelerator_type=AMD_INSTINCT_MI355x, num_gpus=0)
        def f():
            return 7

        assert ray.get(f.remote(), timeout=30) == 7
    finally:
        ray.shutdown()
