"""``Datasink`` (reference: python/ray/data/datasource/datasink.py): on_write_start /
write / on_write_complete / on_write_failed, driven by ``Dataset.write_datasink``."""

from __future__ import annotations

from typing import Any, Iterable, List, Optional

import ray_amd as ray


class Datasink:
    """Subclass and implement ``write(blocks, ctx)``; it runs once per write task (one
    task per dataset block) and its return values reach ``on_write_complete``."""

    def on_write_start(self) -> None:
        pass

    def write(self, blocks: Iterable[dict], ctx: dict) -> Any:
        raise NotImplementedError

    def on_write_complete(self, write_results: List[Any]) -> Any:
        return None

    def on_write_failed(self, error: Exception) -> None:
        pass

    def get_name(self) -> str:
        name = type(self).__name__
        return name[: -len("Datasink")] if name.endswith("Datasink") else name

    @property
    def supports_distributed_writes(self) -> bool:
        return True


@ray.remote
def _sink_write(sink, blk, idx):
    return sink.write([blk], {"task_idx": idx})


def write_datasink(ds, sink: Datasink, ray_remote_args: Optional[dict] = None):
    from ray_amd.data import _executor as X

    sink.on_write_start()
    fn = _sink_write.options(**ray_remote_args) if ray_remote_args else _sink_write
    try:
        if sink.supports_distributed_writes:
            results = ray.get([fn.remote(sink, r, i)
                               for i, (r, _) in enumerate(X.execute(ds._plan))])
        else:  # single writer in the driver
            results = [sink.write([ray.get(r) for r, _ in X.execute(ds._plan)], {"task_idx": 0})]
    except Exception as e:
        sink.on_write_failed(e)
        raise
    return sink.on_write_complete(results)


class DummyOutputDatasink(Datasink):
    """Counts rows and discards them (a sink for benchmarks and tests)."""

    def __init__(self):
        self.num_ok = 0
        self.num_failed = 0
        self.enabled = True

    def write(self, blocks, ctx):
        from ray_amd.data import block as B

        if not self.enabled:
            raise ValueError("disabled")
        return sum(B.num_rows(b) for b in blocks)

    def on_write_complete(self, write_results):
        self.num_ok += 1
        return sum(write_results)

    def on_write_failed(self, error):
        self.num_failed += 1
