"""One thread that drains every worker's stdout / stderr pipe (reference: the per-node
log monitor, python/ray/_private/log_monitor.py, which tails the workers' log files from
one process).

Each worker pipe is registered with a selector (epoll); the pump thread reads whatever is
available, splits it into lines, appends them to the worker's log file under
``<session>/logs`` and forwards them (deduplicated) to the raylet's stdout / stderr, i.e.
the driver's terminal. One thread for the whole node instead of two blocking
``readline`` threads per worker process: a node with hundreds of workers no longer runs
hundreds of Python threads contending for the raylet's GIL.

A pipe is never left undrained: a worker whose 64 KB pipe fills blocks on its next print.
A failed file write (ENOSPC, ...) drops the file copy and keeps forwarding.
"""

from __future__ import annotations

import os
import queue
import selectors
import threading


class _Stream:
    __slots__ = ("fd", "pipe", "file", "out", "pid", "buf")

    def __init__(self, pipe, path, out, pid):
        self.pipe = pipe
        self.fd = pipe.fileno()
        try:
            self.file = open(path, "ab", buffering=0)
        except OSError:
            self.file = None
        self.out = out
        self.pid = pid
        self.buf = b""


class LogPump:
    """``add(pipe, path, out, pid)`` from any thread; the pump thread owns the streams."""

    def __init__(self, dedup):
        self._dedup = dedup
        self._sel = selectors.DefaultSelector()
        self._new: queue.SimpleQueue = queue.SimpleQueue()
        self._rfd, self._wfd = os.pipe()
        os.set_blocking(self._rfd, False)
        self._sel.register(self._rfd, selectors.EVENT_READ, None)
        self._stop = False
        self.streams = 0  # live pipes (tests / diagnostics)
        self._t = threading.Thread(target=self._run, name="log-pump", daemon=True)
        self._t.start()

    def add(self, pipe, path, out, pid):
        self._new.put(_Stream(pipe, path, out, pid))
        try:
            os.write(self._wfd, b"x")
        except OSError:
            pass

    def stop(self):
        self._stop = True
        try:
            os.write(self._wfd, b"x")
        except OSError:
            pass

    def _emit(self, st, line):
        if st.file is not None:
            try:
                st.file.write(line)
            except (ValueError, OSError):
                try:
                    st.file.close()
                except OSError:
                    pass
                st.file = None
        if st.out is None:  # init(log_to_driver=False): files only
            return
        for text in self._dedup.feed(line, st.pid, st.out):
            try:
                st.out.buffer.write(text)
                st.out.flush()
            except (ValueError, OSError, AttributeError):
                pass

    def _close(self, st):
        if st.buf:
            self._emit(st, st.buf)
            st.buf = b""
        try:
            self._sel.unregister(st.fd)
        except (KeyError, ValueError):
            pass
        if st.file is not None:
            try:
                st.file.close()
            except OSError:
                pass
        try:
            st.pipe.close()
        except OSError:
            pass
        self.streams -= 1

    def _run(self):
        while not self._stop:
            for key, _ in self._sel.select(timeout=1.0):
                st = key.data
                if st is None:  # wake pipe: new streams (or stop)
                    try:
                        while os.read(self._rfd, 4096):
                            pass
                    except BlockingIOError:
                        pass
                    while True:
                        try:
                            ns = self._new.get_nowait()
                        except queue.Empty:
                            break
                        os.set_blocking(ns.fd, False)
                        self._sel.register(ns.fd, selectors.EVENT_READ, ns)
                        self.streams += 1
                    continue
                try:
                    data = os.read(st.fd, 65536)
                except BlockingIOError:
                    continue
                except OSError:
                    data = b""
                if not data:  # the worker exited (EOF)
                    self._close(st)
                    continue
                st.buf += data
                *lines, st.buf = st.buf.split(b"\n")
                for ln in lines:
                    self._emit(st, ln + b"\n")
                if len(st.buf) > (1 << 20):  # no newline in 1 MB: pass it on as is
                    self._emit(st, st.buf)
                    st.buf = b""
