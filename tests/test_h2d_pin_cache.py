"""StorePinCache: the object-store chunks a pinned H2D copy touches are registered once,
kept in LRU order and unregistered beyond the byte cap, never dropping a chunk the current
copy needs (CPU test with a recording stand-in for the HIP register calls)."""

from ray_amd._private.h2d import CHUNK, StorePinCache


class _FakeLib:
    def __init__(self, fail_at=None):
        self.reg, self.unreg = [], []
        self.fail_at = fail_at

    def ra_host_register(self, p, n):
        if self.fail_at is not None and p == self.fail_at:
            return 1
        self.reg.append((p, n))
        return 0

    def ra_host_unregister(self, p):
        self.unreg.append(p)
        return 0


def test_chunks_registered_once_and_lru_capped():
    base = 1 << 40
    lib = _FakeLib()
    c = StorePinCache(base, 10 * CHUNK + 123, cap_bytes=3 * CHUNK, lib=lib)
    assert c.ensure(base + 10, 100)                      # chunk 0
    assert c.ensure(base + CHUNK - 5, 10)                # chunks 0, 1
    assert [p for p, _ in lib.reg] == [base, base + CHUNK]
    assert c.ensure(base + 2 * CHUNK, CHUNK)             # chunk 2 (cap reached, no evict)
    assert lib.unreg == []
    assert c.ensure(base + 3 * CHUNK + 1, 1)             # chunk 3: evicts LRU chunk 0
    assert lib.unreg == [base] and c.registered_bytes == 3 * CHUNK
    # a copy wider than the cap keeps all the chunks it needs
    assert c.ensure(base + 4 * CHUNK, 4 * CHUNK)
    assert all(ch in c._chunks for ch in (4, 5, 6, 7))
    # the last chunk is short (store size not a multiple of CHUNK)
    assert c.ensure(base + 10 * CHUNK, 100)
    assert lib.reg[-1] == (base + 10 * CHUNK, 123)


def test_outside_store_and_failures():
    base = 1 << 40
    lib = _FakeLib(fail_at=(1 << 40) + CHUNK)
    c = StorePinCache(base, 4 * CHUNK, cap_bytes=8 * CHUNK, lib=lib)
    assert not c.ensure(base - 1, 10)
    assert not c.ensure(base + 4 * CHUNK, 1)
    assert not c.ensure(base + CHUNK, 10)  # registration failed: copy runs pageable
    assert c.failures == 1 and c.ensure(base, 10)


class _FakeEvent:
    def __init__(self):
        self.done = False
        self.waited = 0

    def query(self):
        return self.done

    def synchronize(self):
        self.waited += 1
        self.done = True


def test_inflight_copy_keeps_chunk_and_source_alive():
    """An async copy's chunks are unregistered only after its event; its source array is
    held until the event completes (the store block may not be recycled under the DMA)."""
    base = 1 << 40
    lib = _FakeLib()
    c = StorePinCache(base, 8 * CHUNK, cap_bytes=2 * CHUNK, lib=lib)
    src = object()
    assert c.ensure(base, 10)
    ev = _FakeEvent()
    c.track(base, 10, ev, src)
    assert c._pending and c._pending[0][1] is src
    assert c.ensure(base + CHUNK, 10) and c.ensure(base + 2 * CHUNK, 10)  # evicts chunk 0
    assert lib.unreg == [base] and ev.waited == 1  # waited for the copy before unregister
    ev2 = _FakeEvent()
    c.track(base + 2 * CHUNK, 10, ev2, object())
    assert len(c._pending) == 1  # the completed copy was released, the new one is held
    c.drain()
    assert ev2.done and not c._pending
