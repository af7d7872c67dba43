"""Parallel iterators over actor-held shards (reference API: python/ray/util/iter.py —
``from_items`` / ``from_range`` / ``from_iterators`` / ``from_actors``, ``ParallelIterator``
with ``for_each``/``filter``/``batch``/``flatten``/``combine``/``local_shuffle``/
``repartition``/``gather_sync``/``gather_async``/``batch_across_shards``/``union``/
``select_shards``/``get_shard``, and the driver-side ``LocalIterator``).

Design: each shard is one ``ParallelIteratorWorker`` actor owning an item generator.
Transformations of a ``ParallelIterator`` are recorded on the driver and shipped to the
shard actors when iteration starts, so they run next to the data (``for_each`` on a GPU
actor runs on that GPU). The driver pulls items in batches (``par_iter_next_batch``) to
amortise the call cost; ``gather_async`` keeps ``num_async`` pulls in flight per shard and
yields whichever shard answers first."""

from __future__ import annotations

import collections
import random
import time

import ray_amd as ray


class _Done:
    pass


_DONE = _Done()


# ============================================================================ shard actor
class ParallelIteratorWorker:
    """Actor mixin: a shard of a ParallelIterator (``from_actors`` accepts any actor whose
    class derives from it)."""

    def __init__(self, item_generator, repeat: bool = False):
        self._make = item_generator
        self._repeat = repeat
        self._transforms = []
        self._it = None
        self._buf = collections.defaultdict(collections.deque)  # slice buffers
        self._pos = 0
        self._exhausted = False

    def _source(self):
        while True:
            src = self._make() if callable(self._make) else self._make
            yield from src
            if not self._repeat:
                return

    def par_iter_init(self, transforms):
        it = iter(self._source())
        for t in transforms:
            it = iter(t(it))
        self._it = it
        self._buf.clear()
        self._pos = 0
        self._exhausted = False
        return True

    def _next(self):
        if self._it is None:
            self.par_iter_init([])
        return next(self._it, _DONE)

    def par_iter_next(self):
        v = self._next()
        if v is _DONE:
            raise StopIteration
        return v

    def par_iter_next_batch(self, max_items: int = 64, batch_ms: float = 0.0):
        """Up to max_items (fewer after batch_ms); (items, exhausted)."""
        out, t0 = [], time.perf_counter()
        while len(out) < max_items:
            v = self._next()
            if v is _DONE:
                return out, True
            out.append(v)
            if batch_ms and (time.perf_counter() - t0) * 1000 >= batch_ms:
                break
        return out, False

    def par_iter_slice_batch(self, step: int, start: int, max_items: int = 64):
        """Items whose position in this shard's stream is = start (mod step);
        (items, exhausted) — exhausted: nothing more will come for this slice."""
        q = self._buf[start]
        while len(q) < max_items and not self._exhausted:
            v = self._next()
            if v is _DONE:
                self._exhausted = True
                break
            self._buf[self._pos % step].append(v)
            self._pos += 1
        out = [q.popleft() for _ in range(min(max_items, len(q)))]
        return out, self._exhausted and not q


_Worker = ray.remote(ParallelIteratorWorker)


# ============================================================================ local iterator
class LocalIterator:
    """Driver-side iterator; transformations compose lazily."""

    def __init__(self, base_iterator, name: str = "LocalIterator"):
        self._base = base_iterator  # zero-arg callable -> iterator
        self.name = name
        self._it = None

    def __iter__(self):
        return self

    def __next__(self):
        if self._it is None:
            self._it = iter(self._base())
        return next(self._it)

    def __repr__(self):
        return f"LocalIterator[{self.name}]"

    def _wrap(self, fn, suffix):
        base = self._base
        return LocalIterator(lambda: fn(iter(base())), f"{self.name}.{suffix}")

    def transform(self, fn):
        return self._wrap(fn, "transform()")

    def for_each(self, fn, max_concurrency: int = 1, resources=None):
        return self._wrap(lambda it: (fn(x) for x in it), "for_each()")

    def filter(self, fn):
        return self._wrap(lambda it: (x for x in it if fn(x)), "filter()")

    def batch(self, n: int):
        return self._wrap(lambda it: _batched(it, n), f"batch({n})")

    def flatten(self):
        return self._wrap(lambda it: (y for x in it for y in x), "flatten()")

    def combine(self, fn):
        return self.for_each(fn).flatten()

    def shuffle(self, shuffle_buffer_size: int, seed: int | None = None):
        return self._wrap(lambda it: _shuffled(it, shuffle_buffer_size, seed),
                          f"shuffle({shuffle_buffer_size})")

    def take(self, n: int) -> list:
        out = []
        for x in self:
            out.append(x)
            if len(out) >= n:
                break
        return out

    def show(self, n: int = 20):
        for x in self.take(n):
            print(x)

    def duplicate(self, n: int) -> list:
        """n iterators over the same stream; items are buffered until every copy saw them."""
        src = iter(self._base())
        queues = [collections.deque() for _ in range(n)]

        def gen(i):
            q = queues[i]
            while True:
                if not q:
                    v = next(src, _DONE)
                    if v is _DONE:
                        return
                    for qq in queues:
                        qq.append(v)
                yield q.popleft()

        return [LocalIterator(lambda i=i: gen(i), f"{self.name}.duplicate[{i}]")
                for i in range(n)]

    def union(self, *others, deterministic: bool = False, round_robin_weights=None):
        its = [self] + list(others)
        w = round_robin_weights or [1] * len(its)

        def gen():
            live = [iter(i._base()) for i in its]
            active = list(range(len(live)))
            while active:
                for k in list(active):
                    for _ in range(w[k] if w[k] != "*" else 1 << 30):
                        v = next(live[k], _DONE)
                        if v is _DONE:
                            active.remove(k)
                            break
                        yield v

        return LocalIterator(gen, f"LocalUnion[{', '.join(i.name for i in its)}]")

    def zip_with_source_actor(self):
        return self._wrap(lambda it: it, "zip_with_source_actor()")


def _batched(it, n):
    b = []
    for x in it:
        b.append(x)
        if len(b) == n:
            yield b
            b = []
    if b:
        yield b


def _shuffled(it, size, seed):
    rng = random.Random(seed)
    buf = []
    for x in it:
        buf.append(x)
        if len(buf) >= size:
            yield buf.pop(rng.randrange(len(buf)))
    rng.shuffle(buf)
    yield from buf


# ============================================================================ parallel iterator
class ParallelIterator:
    def __init__(self, actors: list, name: str, transforms: list | None = None,
                 pulls: list | None = None):
        self.actors = list(actors)
        self.name = name
        self._transforms = list(transforms or [])
        # per shard: how the driver pulls ("next" or ("slice", step, start, sources))
        self._pulls = pulls

    def __repr__(self):
        return f"ParallelIterator[{self.name}]"

    __str__ = __repr__

    def __iter__(self):
        raise TypeError("You must use it.gather_sync() or it.gather_async() to iterate "
                        "over the results of a ParallelIterator.")

    def _with(self, t, suffix):
        return ParallelIterator(self.actors, f"{self.name}.{suffix}", self._transforms + [t],
                                self._pulls)

    def transform(self, fn):
        return self._with(fn, "transform()")

    def for_each(self, fn, max_concurrency: int = 1, resources=None):
        return self._with(lambda it: (fn(x) for x in it), "for_each()")

    def filter(self, fn):
        return self._with(lambda it: (x for x in it if fn(x)), "filter()")

    def batch(self, n: int):
        return self._with(lambda it: _batched(it, n), f"batch({n})")

    def flatten(self):
        return self._with(lambda it: (y for x in it for y in x), "flatten()")

    def combine(self, fn):
        return self.for_each(fn).flatten()

    def local_shuffle(self, shuffle_buffer_size: int, seed: int | None = None):
        return self._with(lambda it: _shuffled(it, shuffle_buffer_size, seed),
                          f"local_shuffle({shuffle_buffer_size})")

    def num_shards(self) -> int:
        return len(self.actors)

    # --- pulling -------------------------------------------------------------------
    def _init_shards(self):
        ray.get([a.par_iter_init.remote(self._transforms) for a in self.actors])

    def _shard_gen(self, i, batch: int = 64):
        a = self.actors[i]
        while True:
            items, done = ray.get(a.par_iter_next_batch.remote(batch))
            yield from items
            if done:
                return

    def gather_sync(self) -> LocalIterator:
        """Round-robin, one item per shard in turn (deterministic order)."""
        def gen():
            self._init_shards()
            gens = [self._shard_gen(i, 1) for i in range(len(self.actors))]
            active = list(range(len(gens)))
            while active:
                for k in list(active):
                    v = next(gens[k], _DONE)
                    if v is _DONE:
                        active.remove(k)
                    else:
                        yield v

        return LocalIterator(gen, f"{self.name}.gather_sync()")

    def batch_across_shards(self) -> LocalIterator:
        def gen():
            self._init_shards()
            gens = [self._shard_gen(i, 1) for i in range(len(self.actors))]
            while True:
                row = [next(g, _DONE) for g in gens]
                row = [v for v in row if v is not _DONE]
                if not row:
                    return
                yield row

        return LocalIterator(gen, f"{self.name}.batch_across_shards()")

    def gather_async(self, batch_ms: float = 0, num_async: int = 1) -> LocalIterator:
        """Items in arrival order; num_async batched pulls in flight per shard."""
        if num_async < 1:
            raise ValueError("num_async must be positive")

        def gen():
            self._init_shards()
            inflight = {}
            for a in self.actors:
                for _ in range(num_async):
                    inflight[a.par_iter_next_batch.remote(64, batch_ms)] = a
            done_actors = set()
            while inflight:
                ready, _ = ray.wait(list(inflight), num_returns=1)
                a = inflight.pop(ready[0])
                items, done = ray.get(ready[0])
                yield from items
                if done:
                    done_actors.add(a)
                elif a not in done_actors:
                    inflight[a.par_iter_next_batch.remote(64, batch_ms)] = a

        return LocalIterator(gen, f"{self.name}.gather_async()")

    def take(self, n: int) -> list:
        return self.gather_sync().take(n)

    def show(self, n: int = 20):
        self.gather_sync().show(n)

    def union(self, other: "ParallelIterator") -> "ParallelIterator":
        if self._transforms != other._transforms and (self._transforms or other._transforms):
            # transforms are per-iterator: bake each side's chain into its own shards
            a = from_iterators([_ShardStream(self, i) for i in range(self.num_shards())])
            b = from_iterators([_ShardStream(other, i) for i in range(other.num_shards())])
            return ParallelIterator(a.actors + b.actors, f"ParallelUnion[{self}, {other}]")
        return ParallelIterator(self.actors + other.actors, f"ParallelUnion[{self}, {other}]",
                                self._transforms)

    def select_shards(self, shards_to_keep) -> "ParallelIterator":
        keep = [self.actors[i] for i in shards_to_keep]
        return ParallelIterator(keep, f"{self.name}.select_shards({len(keep)} total)",
                                self._transforms)

    def shards(self) -> list:
        return [self.get_shard(i) for i in range(self.num_shards())]

    def get_shard(self, shard_index: int, batch_ms: float = 0, num_async: int = 1
                  ) -> LocalIterator:
        def gen():
            a = self.actors[shard_index]
            ray.get(a.par_iter_init.remote(self._transforms))
            yield from self._shard_gen(shard_index)

        return LocalIterator(gen, f"{self.name}.shard[{shard_index}]")

    def repartition(self, num_partitions: int, batch_ms: float = 0) -> "ParallelIterator":
        """num_partitions new shards; partition p receives every item at position = p
        (mod num_partitions) of each source shard's stream (sources buffer per slice)."""
        ray.get([a.par_iter_init.remote(self._transforms) for a in self.actors])
        workers = [_Worker.remote(_SliceStream(self.actors, num_partitions, p))
                   for p in range(num_partitions)]
        return ParallelIterator(workers, f"{self.name}.repartition({num_partitions})")


class _SliceStream:
    """Picklable item factory of one repartitioned shard."""

    def __init__(self, sources, step, start):
        self.sources, self.step, self.start = list(sources), step, start

    def __call__(self):
        live = list(self.sources)
        while live:
            for a in list(live):
                got, done = ray.get(a.par_iter_slice_batch.remote(self.step, self.start))
                yield from got
                if done:
                    live.remove(a)


class _ShardStream:
    """Picklable zero-arg factory streaming one shard of another ParallelIterator."""

    def __init__(self, pit, i):
        self.actor = pit.actors[i]
        self.transforms = pit._transforms

    def __call__(self):
        ray.get(self.actor.par_iter_init.remote(self.transforms))
        while True:
            items, done = ray.get(self.actor.par_iter_next_batch.remote(64))
            yield from items
            if done:
                return


# ============================================================================ constructors
def from_items(items: list, num_shards: int = 2, repeat: bool = False) -> ParallelIterator:
    shards = [[] for _ in range(num_shards)]
    for i, x in enumerate(items):
        shards[i % num_shards].append(x)
    name = f"from_items[{type(items[0]).__name__ if items else 'None'}, {len(items)}, " \
           f"shards={num_shards}{', repeat=True' if repeat else ''}]"
    return from_iterators(shards, repeat=repeat, name=name)


def from_range(n: int, num_shards: int = 2, repeat: bool = False) -> ParallelIterator:
    gens = []
    per = n // num_shards
    for i in range(num_shards):
        start = i * per
        end = n if i == num_shards - 1 else start + per
        gens.append(range(start, end))
    return from_iterators(gens, repeat=repeat,
                          name=f"from_range[{n}, shards={num_shards}"
                               f"{', repeat=True' if repeat else ''}]")


def from_iterators(generators: list, repeat: bool = False, name: str | None = None
                   ) -> ParallelIterator:
    actors = [_Worker.remote(g, repeat) for g in generators]
    return ParallelIterator(actors, name or f"from_iterators[shards={len(generators)}"
                                            f"{', repeat=True' if repeat else ''}]")


def from_actors(actors: list, name: str | None = None) -> ParallelIterator:
    return ParallelIterator(actors, name or f"from_actors[shards={len(actors)}]")


__all__ = ["ParallelIterator", "LocalIterator", "ParallelIteratorWorker", "from_items",
           "from_range", "from_iterators", "from_actors"]
