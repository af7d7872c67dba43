"""Backend plug-in interface (reference: python/ray/train/backend.py)."""

from __future__ import annotations


class BackendConfig:
    @property
    def backend_cls(self):
        return Backend

    def __repr__(self):
        return f"{type(self).__name__}()"


class Backend:
    share_cuda_visible_devices: bool = False

    def on_start(self, worker_group, backend_config):
        pass

    def on_shutdown(self, worker_group, backend_config):
        pass

    def on_training_start(self, worker_group, backend_config):
        pass
