"""Dataset iteration + Train ingest (reference: python/ray/data/iterator.py,
_internal/iterator/stream_split_iterator.py, _internal/block_batching/*).

``iter_torch_batches(device="cuda")`` on MI355X: each numpy batch (a zero-copy
view of the shared-memory block) is copied ONCE into a reusable pinned host
buffer and moved to HBM with a non-blocking H2D on a side stream, one batch
ahead of the consumer; the consumer's stream waits on an event, so the DMA
overlaps the training step."""

from __future__ import annotations

import collections

import numpy as np

import ray_amd as ray
from ray_amd._native import _core

from . import block as B


def _fetch(ref):
    if isinstance(ref, tuple):  # (block ref, start row, end row): an equal split's share
        r0, a, b = ref
        return B.slice_block(ray.get(r0), a, b)
    return ray.get(ref)


def _prefetched_blocks(block_refs, depth):
    """Blocks of ``block_refs`` fetched (ray.get + deserialise) ``depth`` ahead on a
    background thread, so the fetch of the next block overlaps the consumer's work on this
    one (reference: iter_batches(prefetch_batches=...)). depth 0: fetched inline."""
    if depth <= 0:
        for ref in block_refs:
            yield _fetch(ref)
        return
    import queue
    import threading

    q = queue.Queue(maxsize=depth)
    stop = threading.Event()
    _END = object()

    def run():
        try:
            for ref in block_refs:
                blk = _fetch(ref)
                while not stop.is_set():
                    try:
                        q.put((True, blk), timeout=0.2)
                        break
                    except queue.Full:
                        continue
                if stop.is_set():
                    return
            q.put((True, _END))
        except BaseException as e:  # noqa: BLE001  (re-raised in the consumer)
            q.put((False, e))

    t = threading.Thread(target=run, daemon=True, name="ray_amd-data-prefetch")
    t.start()
    try:
        while True:
            ok, item = q.get()
            if not ok:
                raise item
            if item is _END:
                return
            yield item
    finally:
        stop.set()


def batch_blocks(block_refs, batch_size, batch_format, drop_last, shuffle_buffer, seed,
                 prefetch=0):
    rng = np.random.default_rng(seed)
    buf = []
    buffered = 0
    bs = None if batch_size in (None, "default") else int(batch_size)
    fmt = "numpy" if batch_format in ("default", None) else batch_format

    def emit(blk):
        return B.to_batch(blk, fmt)

    for blk in _prefetched_blocks(block_refs, prefetch):
        if B.num_rows(blk) == 0:
            continue
        if bs is None:
            yield emit(blk)
            continue
        buf.append(blk)
        buffered += B.num_rows(blk)
        min_buf = bs if not shuffle_buffer else max(bs, shuffle_buffer)
        while buffered >= min_buf:
            cat = B.concat(buf)
            if shuffle_buffer:
                cat = B.take_idx(cat, rng.permutation(B.num_rows(cat)))
            out = B.slice_block(cat, 0, bs)
            rest = B.slice_block(cat, bs, B.num_rows(cat))
            buf = [rest] if B.num_rows(rest) else []
            buffered = B.num_rows(rest)
            yield emit(out)
    if buf and bs is not None:
        cat = B.concat(buf)
        if shuffle_buffer:
            cat = B.take_idx(cat, rng.permutation(B.num_rows(cat)))
        n = B.num_rows(cat)
        for s in range(0, n, bs):
            part = B.slice_block(cat, s, min(n, s + bs))
            if drop_last and B.num_rows(part) < bs:
                break
            yield emit(part)


def _resolve_device(device):
    import torch

    if device == "auto":
        from ray_amd.train._internal import session as S

        if S._get_session(required=False) is not None and torch.cuda.is_available():
            from ray_amd.train.torch import get_device

            return get_device()
        return torch.device("cpu")
    return torch.device(device) if device is not None else torch.device("cpu")


def _same_device(a, b):
    import torch

    if a.type != b.type:
        return False
    if a.type != "cuda":
        return True
    ia = a.index if a.index is not None else torch.cuda.current_device()
    ib = b.index if b.index is not None else torch.cuda.current_device()
    return ia == ib


def torch_batches(batches, dtypes, device, collate_fn, pin_memory=True):
    import torch

    dev = _resolve_device(device)
    if collate_fn is not None:
        for b in batches:
            yield collate_fn(b)
        return

    def to_tensors(b):
        out = {}
        for k, v in b.items():
            if B._is_tensor(v):  # device block column: already a tensor
                t = v.to(dev)
                if dtypes is not None:
                    dt = dtypes.get(k) if isinstance(dtypes, dict) else dtypes
                    if dt is not None:
                        t = t.to(dt)
                out[k] = t
                continue
            if v.dtype == object:
                out[k] = list(v)
                continue
            t = torch.from_numpy(np.array(v, copy=not v.flags.writeable))
            if dtypes is not None:
                dt = dtypes.get(k) if isinstance(dtypes, dict) else dtypes
                if dt is not None:
                    t = t.to(dt)
            out[k] = t
        return out

    if dev.type != "cuda":
        for b in batches:
            yield to_tensors(b)
        return
    stream = torch.cuda.Stream(dev)
    # two pinned staging sets (ping-pong): set s is refilled only after the H2D that
    # read it two batches ago has retired (its event), so host copies never race DMA
    pinned = [{}, {}]
    fence = [None, None]
    slot = [0]

    def stage(b):
        s = slot[0]
        slot[0] ^= 1
        if fence[s] is not None:
            fence[s].synchronize()
        out = {}
        with torch.cuda.stream(stream):
            for k, v in b.items():
                if B._is_tensor(v):
                    # HBM-resident block: no copy on the same GPU, a D2D/H2D otherwise
                    t = v if _same_device(v.device, dev) else v.to(dev, non_blocking=True)
                    dt = dtypes.get(k) if isinstance(dtypes, dict) else dtypes
                    out[k] = t if dt is None else t.to(dt)
                    continue
                if v.dtype == object:
                    out[k] = list(v)
                    continue
                v = np.ascontiguousarray(v)
                key = (k, v.shape, v.dtype.str)
                buf = pinned[s].get(key)
                if buf is None:
                    buf = torch.empty(v.shape, dtype=torch.from_numpy(np.empty(0, v.dtype)).dtype,
                                      pin_memory=pin_memory)
                    pinned[s][key] = buf
                # one threaded copy, GIL released, straight from the (read-only) store
                # view into the pinned buffer
                _core.copy_into(buf.numpy().reshape(-1).view(np.uint8),
                                v.reshape(-1).view(np.uint8))
                t = buf.to(dev, non_blocking=True)
                if dtypes is not None:
                    dt = dtypes.get(k) if isinstance(dtypes, dict) else dtypes
                    if dt is not None:
                        t = t.to(dt)
                out[k] = t
            ev = torch.cuda.Event()
            ev.record(stream)
        fence[s] = ev
        return out, ev

    def hand_over(out, ev):
        cur = torch.cuda.current_stream(dev)
        cur.wait_event(ev)
        for t in out.values():
            if isinstance(t, torch.Tensor):
                t.record_stream(cur)  # allocated on the copy stream, consumed on `cur`
        return out

    nxt = None
    for b in batches:
        cur = stage(b)
        if nxt is not None:
            yield hand_over(*nxt)
        nxt = cur
    if nxt is not None:
        yield hand_over(*nxt)


class DataIterator:
    def __init__(self, ds):
        self._ds = ds

    def iter_batches(self, **kw):
        return self._ds.iter_batches(**kw)

    def iter_torch_batches(self, **kw):
        return self._ds.iter_torch_batches(**kw)

    def iter_rows(self, **kw):
        return self._ds.iter_rows(**kw)

    def materialize(self):
        return self._ds.materialize()

    def stats(self):
        return self._ds.stats()

    def schema(self):
        """Schema of the rows this iterator yields (the dataset's)."""
        return self._ds.schema()

    def to_torch(self, *, label_column=None, feature_columns=None, batch_size=1,
                 label_column_dtype=None, feature_column_dtypes=None, **kw):
        """A torch ``IterableDataset`` of (features, label) batches (reference: the
        deprecated ``DataIterator.to_torch``)."""
        import torch

        it = self

        class _Iterable(torch.utils.data.IterableDataset):
            def __iter__(self):
                for b in it.iter_torch_batches(batch_size=batch_size, **kw):
                    y = b.pop(label_column) if label_column else None
                    cols = feature_columns or sorted(b)
                    x = torch.stack([b[c].float() if feature_column_dtypes is None
                                     else b[c].to(feature_column_dtypes) for c in cols], 1) \
                        if isinstance(cols, list) else b[cols]
                    if y is not None and label_column_dtype is not None:
                        y = y.to(label_column_dtype)
                    yield (x, y) if y is not None else x

        return _Iterable()

    def to_tf(self, feature_columns, label_columns, **kw):
        from ray_amd.data import integrations

        return integrations.to_tf(self, feature_columns, label_columns, **kw)

    def iter_tf_batches(self, **kw):
        from ray_amd.data import integrations

        return integrations.iter_tf_batches(self, **kw)


class SplitCoordinator:
    """Actor that runs ONE streaming execution and deals its blocks to n consumers
    (reference: stream_split_iterator.SplitCoordinator)."""

    def __init__(self, plan, n, equal):
        self.plan = plan
        self.n = n
        self.equal = equal
        self.epoch = -1
        self._start()

    def _start(self):
        from . import _executor as X

        self.epoch += 1
        self.gen = X.execute(self.plan)
        self.queues = [collections.deque() for _ in range(self.n)]
        self.rows = [0] * self.n
        self.carry = collections.deque()
        self.carry_rows = 0
        self.done = False
        self.finished = [False] * self.n
        self.served = [0] * self.n  # requests answered per consumer this epoch

    def next_block(self, i, epoch, seq=None):
        """Consumer ``i``'s ``seq``-th block of ``epoch`` (None: its share is exhausted).

        The actor serves requests on several threads, so a consumer's prefetched requests
        can arrive out of order: each is answered in ``seq`` order per consumer (request
        k waits for k-1), or a later request could take the block an earlier one should
        have returned while the earlier one reports the end of the epoch. A consumer that
        starts epoch e+1 while others still read epoch e waits for them (the reference
        coordinator's epoch barrier) instead of getting an empty epoch; waits are bounded
        so a consumer that never comes back cannot wedge the others forever."""
        import threading
        import time

        if not hasattr(self, "_cond"):
            self._cond = threading.Condition()
        with self._cond:
            deadline = time.monotonic() + 600.0
            while True:
                if epoch < self.epoch:  # a prefetch request left over from a finished epoch
                    return None
                if epoch > self.epoch and all(self.finished):
                    self._start()
                    continue
                if epoch == self.epoch and (seq is None or seq == self.served[i]):
                    break
                if time.monotonic() > deadline:
                    raise TimeoutError(f"streaming_split consumer {i} waited 600 s for "
                                       f"epoch {epoch} (the coordinator is at {self.epoch})")
                self._cond.wait(timeout=1.0)
            r = self._next_block(i, epoch)
            self.served[i] += 1
            self._cond.notify_all()
            return r

    def _next_block(self, i, epoch):
        while not self.queues[i]:
            if self.done:
                self.finished[i] = True
                return None
            try:
                ref, meta = next(self.gen)
            except StopIteration:
                self.done = True
                continue
            if self.equal:
                self._deal_equal(ref, meta["num_rows"] if meta else 0)
                continue
            j = sum(len(q) for q in self.queues) % self.n
            self.queues[j].append(ref)
            self.rows[j] += meta["num_rows"] if meta else 0
        return [self.queues[i].popleft()]

    def _deal_equal(self, ref, rows):
        """equal=True: every consumer gets floor(rows / n) rows of each block (a row range
        of the same block ref, sliced zero-copy by the consumer); the < n leftover rows of
        each block join a carry pool that is dealt the same way once it holds n rows, and
        is dropped at the end — so all consumers receive exactly the same number of rows."""
        n = self.n
        per = rows // n
        if per:
            for j in range(n):
                self.queues[j].append((ref, j * per, (j + 1) * per))
                self.rows[j] += per
        if rows - per * n:
            self.carry.append((ref, per * n, rows))
            self.carry_rows += rows - per * n
        while self.carry_rows >= n:
            for j in range(n):  # one row from the carry pool to each consumer
                r, a, b = self.carry[0]
                self.queues[j].append((r, a, a + 1))
                self.rows[j] += 1
                if a + 1 == b:
                    self.carry.popleft()
                else:
                    self.carry[0] = (r, a + 1, b)
            self.carry_rows -= n


class StreamSplitIterator(DataIterator):
    def __init__(self, coord, index):
        self._coord = coord
        self._index = index
        self._epoch = 0

    # next_block requests kept in flight per consumer: the coordinator round trip (and
    # its wait for the executor) overlaps the consumer's work on the previous block
    PREFETCH_BLOCKS = 2

    def _blocks(self):
        ep = self._epoch
        self._epoch += 1
        seq = 0
        window = collections.deque()
        for _ in range(self.PREFETCH_BLOCKS):
            window.append(self._coord.next_block.remote(self._index, ep, seq))
            seq += 1
        while window:
            r = ray.get(window.popleft())
            if r is None:
                for x in window:  # the shard is exhausted: the rest answer None too
                    ray.get(x)
                return
            window.append(self._coord.next_block.remote(self._index, ep, seq))
            seq += 1
            yield r[0]

    def iter_batches(self, *, batch_size=256, batch_format="default", drop_last=False,
                     local_shuffle_buffer_size=None, local_shuffle_seed=None, prefetch_batches=1,
                     **kw):
        return batch_blocks(self._blocks(), batch_size, batch_format, drop_last,
                            local_shuffle_buffer_size, local_shuffle_seed,
                            prefetch=prefetch_batches)

    def iter_rows(self, **kw):
        for ref in self._blocks():
            if isinstance(ref, tuple):
                yield from B.to_rows(B.slice_block(ray.get(ref[0]), ref[1], ref[2]))
            else:
                yield from B.to_rows(ray.get(ref))

    def iter_torch_batches(self, *, batch_size=256, dtypes=None, device="auto", collate_fn=None,
                           drop_last=False, local_shuffle_buffer_size=None,
                           local_shuffle_seed=None, prefetch_batches=1, **kw):
        return torch_batches(self.iter_batches(batch_size=batch_size, drop_last=drop_last,
                                               local_shuffle_buffer_size=local_shuffle_buffer_size,
                                               local_shuffle_seed=local_shuffle_seed,
                                               prefetch_batches=prefetch_batches),
                             dtypes, device, collate_fn)

    def __reduce__(self):
        return (StreamSplitIterator, (self._coord, self._index))
