"""Accelerator type constants and node detection (reference:
python/ray/util/accelerators/accelerators.py, python/ray/_private/accelerators/amd_gpu.py).

``@ray.remote(accelerator_type=AMD_INSTINCT_MI355X)`` requests the node resource
``accelerator_type:AMD-Instinct-MI355X`` that the raylet advertises (0.001 per request).
Detection reads the KFD topology (no HIP initialisation, no amd-smi dependency):
``gfx_target_version`` identifies the CDNA generation and the PCI ``device_id``
distinguishes the SKUs of one generation.
"""

from __future__ import annotations

import os

AMD_INSTINCT_MI100 = "AMD-Instinct-MI100"
AMD_INSTINCT_MI210 = "AMD-Instinct-MI210"
AMD_INSTINCT_MI250x = "AMD-Instinct-MI250X"
AMD_INSTINCT_MI250 = "AMD-Instinct-MI250X-MI250"
AMD_INSTINCT_MI300x = "AMD-Instinct-MI300X-OAM"
AMD_INSTINCT_MI300A = "AMD-Instinct-MI300A"
AMD_INSTINCT_MI325x = "AMD-Instinct-MI325X-OAM"
AMD_INSTINCT_MI350x = "AMD-Instinct-MI350X"
AMD_INSTINCT_MI355x = "AMD-Instinct-MI355X"

AMD_RADEON_R9_200_HD_7900 = "AMD-Radeon-R9-200-HD-7900"
AMD_RADEON_HD_7900 = "AMD-Radeon-HD-7900"
# other vendors' type names (API parity: user code may name them; no such node here)
NVIDIA_TESLA_V100 = "V100"
NVIDIA_TESLA_P100 = "P100"
NVIDIA_TESLA_T4 = "T4"
NVIDIA_TESLA_P4 = "P4"
NVIDIA_TESLA_K80 = "K80"
NVIDIA_TESLA_A10G = "A10G"
NVIDIA_L4 = "L4"
NVIDIA_A100 = "A100"
NVIDIA_A100_40G = "A100-40G"
NVIDIA_A100_80G = "A100-80G"
NVIDIA_H100 = "H100"
INTEL_MAX_1550 = "Intel-GPU-Max-1550"
INTEL_MAX_1100 = "Intel-GPU-Max-1100"
INTEL_GAUDI = "Intel-GAUDI"
AWS_NEURON_CORE = "aws-neuron-core"
GOOGLE_TPU_V2 = "TPU-V2"
GOOGLE_TPU_V3 = "TPU-V3"
GOOGLE_TPU_V4 = "TPU-V4"
GOOGLE_TPU_V5P = "TPU-V5P"
GOOGLE_TPU_V5LITEPOD = "TPU-V5LITEPOD"
GOOGLE_TPU_V6E = "TPU-V6E"

# PCI device ids (amdgpu.ids) -> accelerator type
_DEVICE_IDS = {
    0x738C: AMD_INSTINCT_MI100, 0x738E: AMD_INSTINCT_MI100,
    0x740F: AMD_INSTINCT_MI210, 0x7408: AMD_INSTINCT_MI250x, 0x740C: AMD_INSTINCT_MI250,
    0x74A1: AMD_INSTINCT_MI300x, 0x74A0: AMD_INSTINCT_MI300A, 0x74A5: AMD_INSTINCT_MI325x,
    0x75A0: AMD_INSTINCT_MI350x, 0x75A3: AMD_INSTINCT_MI355x,
}
# gfx_target_version (KFD) -> generation name when the device id is unknown
_GFX = {90008: AMD_INSTINCT_MI100, 90010: AMD_INSTINCT_MI250x, 90402: AMD_INSTINCT_MI300x,
        90500: AMD_INSTINCT_MI355x}

_KFD = "/sys/class/kfd/kfd/topology/nodes"


def _props(path):
    out = {}
    try:
        with open(path) as f:
            for line in f:
                k, _, v = line.partition(" ")
                try:
                    out[k] = int(v)
                except ValueError:
                    pass
    except OSError:
        pass
    return out


def detect_accelerator_type(kfd_root: str = _KFD) -> str | None:
    """Accelerator type of the node's GPUs (the first GPU node in the KFD topology)."""
    try:
        nodes = sorted(os.listdir(kfd_root), key=lambda x: int(x) if x.isdigit() else 0)
    except OSError:
        return None
    for n in nodes:
        p = _props(os.path.join(kfd_root, n, "properties"))
        if p.get("simd_count", 0) <= 0:
            continue
        t = _DEVICE_IDS.get(p.get("device_id", -1))
        if t:
            return t
        gfx = p.get("gfx_target_version")
        if gfx in _GFX:
            return _GFX[gfx]
        if gfx:
            return f"AMD-Instinct-gfx{gfx // 10000}{(gfx // 100) % 100:x}{gfx % 100:x}"
    return None


__all__ = [k for k in list(globals()) if k.startswith("AMD_")] + ["detect_accelerator_type"]
