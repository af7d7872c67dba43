"""``ray_amd.client(address).namespace(...).env(...).connect()`` (reference:
python/ray/client_builder.py). ``address`` "ray://host:port" goes through the Ray Client
server (util/client); "auto" / None / a session address attaches a regular driver."""

from __future__ import annotations

from dataclasses import dataclass, field


@dataclass
class ClientContext:
    dashboard_url: str | None = None
    python_version: str = ""
    ray_version: str = ""
    ray_commit: str = ""
    protocol_version: str | None = None
    _num_clients: int = 1
    _extra: dict = field(default_factory=dict)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.disconnect()

    def disconnect(self):
        import ray_amd

        ray_amd.shutdown()

    def __getitem__(self, key):
        return getattr(self, key)


class ClientBuilder:
    def __init__(self, address: str | None = None):
        self.address = address
        self._namespace = None
        self._runtime_env = None
        self._init_kwargs: dict = {}

    def namespace(self, namespace: str) -> "ClientBuilder":
        self._namespace = namespace
        return self

    def env(self, env: dict) -> "ClientBuilder":
        self._runtime_env = env
        return self

    def _init_args(self, **kwargs) -> "ClientBuilder":
        self._init_kwargs.update(kwargs)
        return self

    def connect(self) -> ClientContext:
        import platform

        import ray_amd

        addr = self.address
        if addr is not None and "://" not in addr and addr != "auto" and ":" in addr:
            addr = "ray://" + addr
        ray_amd.init(address=addr, namespace=self._namespace, runtime_env=self._runtime_env,
                     **self._init_kwargs)
        return ClientContext(python_version=platform.python_version(),
                             ray_version=ray_amd.__version__)


def client(address: str | None = None, _deprecation_warn_enabled: bool = True) -> ClientBuilder:
    return ClientBuilder(address)
