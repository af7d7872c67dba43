"""Driver-terminal deduplication of worker log lines (reference:
python/ray/_private/ray_logging.py LogDeduplicator, RAY_DEDUP_LOGS).

A line is keyed by its words that contain no digits (pids, ids, counters, timings differ
between workers). The first occurrence of a key is printed at once; further occurrences
from OTHER worker processes within ``RAY_DEDUP_LOGS_AGG_WINDOW_S`` (default 5 s) are
counted (one process repeating itself is printed as is), and when the window closes the
latest one is printed once with ``[repeated Nx across cluster]``. The per-worker
log files under ``<session>/logs`` always keep every line; ``RAY_DEDUP_LOGS=0`` turns the
terminal deduplication off. Lines matching ``RAY_DEDUP_LOGS_SKIP_REGEX`` or
``RAY_DEDUP_LOGS_ALLOW_REGEX`` are dropped / never deduplicated, as in the reference."""

from __future__ import annotations

import os
import re
import threading
import time

_NUMBERS = re.compile(r"\d|0x[0-9a-fA-F]")


def canonicalise(line: str) -> str:
    return " ".join(w for w in line.split() if not _NUMBERS.search(w))


class LogDeduplicator:
    def __init__(self, window_s: float = 5.0, enabled: bool = True, allow_re=None,
                 skip_re=None, background: bool = True):
        self.window_s = window_s
        self.background = background  # a thread prints finished windows
        self.enabled = enabled
        self.allow_re = re.compile(allow_re) if allow_re else None
        self.skip_re = re.compile(skip_re) if skip_re else None
        self.lock = threading.Lock()
        self.state = {}  # (out, key) -> [first_ts, count, last_line, sources]
        self._flusher = None

    @classmethod
    def from_env(cls):
        return cls(float(os.environ.get("RAY_DEDUP_LOGS_AGG_WINDOW_S", "5")),
                   os.environ.get("RAY_DEDUP_LOGS", "1") != "0",
                   os.environ.get("RAY_DEDUP_LOGS_ALLOW_REGEX"),
                   os.environ.get("RAY_DEDUP_LOGS_SKIP_REGEX"))

    def feed(self, raw: bytes, source, out) -> list:
        """Lines (bytes) to write now for one incoming worker line."""
        try:
            line = raw.decode("utf-8", "replace")
        except Exception:  # noqa: BLE001
            return [raw]
        if self.skip_re is not None and self.skip_re.search(line):
            return []
        if not self.enabled or (self.allow_re is not None and self.allow_re.search(line)):
            return [raw]
        key = canonicalise(line)
        if not key:
            return [raw]
        now = time.monotonic()
        with self.lock:
            st = self.state.get((out, key))
            if st is None or now - st[0] > self.window_s:
                self.state[(out, key)] = [now, 0, line, {source}]
                self._ensure_flusher()
                return [raw]
            st[3].add(source)
            if len(st[3]) == 1:  # one process repeating itself is not deduplicated
                return [raw]
            st[1] += 1
            st[2] = line
            return []

    def _ensure_flusher(self):
        if self._flusher is None and self.background:
            self._flusher = threading.Thread(target=self._flush_loop, daemon=True,
                                             name="log-dedup")
            self._flusher.start()

    def flush(self, force: bool = False) -> list:
        """(out, text) pairs of finished windows with repeats to report."""
        now = time.monotonic()
        ready = []
        with self.lock:
            for k, st in list(self.state.items()):
                if force or now - st[0] > self.window_s:
                    del self.state[k]
                    if st[1]:
                        text = st[2].rstrip("\n")
                        ready.append((k[0], f"{text} [repeated {st[1]}x across cluster]\n"))
        return ready

    def _flush_loop(self):
        while True:
            time.sleep(min(1.0, self.window_s / 2 or 0.5))
            for out, text in self.flush():
                try:
                    out.write(text)
                    out.flush()
                except (ValueError, OSError):
                    pass
