"""``ray.train.util.DummyTrainer`` (reference: python/ray/air/util/check_ingest.py): a
trainer that only consumes its "train" dataset shard, to measure the ingest pipeline
(blocks per second into each worker, first-batch latency) without a model."""

from __future__ import annotations

import time

from ray_amd.train.data_parallel_trainer import DataParallelTrainer


def _ingest_loop(config):
    from ray_amd import train

    shard = train.get_dataset_shard("train")
    rows = batches = 0
    first = None
    t0 = time.perf_counter()
    for _ in range(int(config.get("num_epochs", 1))):
        for b in shard.iter_batches(batch_size=config.get("batch_size"),
                                    prefetch_batches=config.get("prefetch_batches", 1)):
            if first is None:
                first = time.perf_counter() - t0
            batches += 1
            rows += len(next(iter(b.values()))) if isinstance(b, dict) else len(b)
    dt = time.perf_counter() - t0
    train.report({"rows_read": rows, "batches_read": batches,
                  "rows_per_second": rows / max(dt, 1e-9),
                  "time_to_first_batch_s": first, "ingest_time_s": dt})


class DummyTrainer(DataParallelTrainer):
    """Reads ``datasets["train"]`` for ``num_epochs`` on every worker and reports the
    ingest throughput."""

    def __init__(self, *args, scaling_config=None, num_epochs: int = 1,
                 prefetch_batches: int = 1, batch_size: int | None = 4096, **kwargs):
        kwargs.pop("train_loop_per_worker", None)
        super().__init__(_ingest_loop, *args, scaling_config=scaling_config,
                         train_loop_config={"num_epochs": num_epochs,
                                            "prefetch_batches": prefetch_batches,
                                            "batch_size": batch_size}, **kwargs)


__all__ = ["DummyTrainer"]
