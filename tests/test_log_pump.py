"""LogPump (ray_amd/_private/log_pump.py): one selector thread drains every worker's
stdout/stderr pipe into its log file and forwards the lines to the driver stream, in
order per pipe, including a last line without a newline and a burst larger than the pipe
buffer (a writer must never block on a full pipe)."""

import io
import subprocess
import sys
import threading

from ray_amd._private.log_pump import LogPump


class _Dedup:  # pass-through stand-in for LogDeduplicator
    def feed(self, line, pid, out):
        return [line]


class _Out:
    def __init__(self):
        self.buffer = io.BytesIO()
        self.lock = threading.Lock()

    def flush(self):
        pass


def test_one_thread_drains_many_pipes(tmp_path):
    before = threading.active_count()
    pump = LogPump(_Dedup())
    out = _Out()
    procs = []
    code = ("import sys\n"
            "for i in range(2000): print(f'{sys.argv[1]} line {i} ' + 'x' * 60)\n"
            "sys.stdout.write('tail-no-newline')\n")
    for k in range(12):
        p = subprocess.Popen([sys.executable, "-c", code, f"w{k}"], stdout=subprocess.PIPE,
                             stderr=subprocess.PIPE)
        pump.add(p.stdout, str(tmp_path / f"w{k}.out"), out, p.pid)
        pump.add(p.stderr, str(tmp_path / f"w{k}.err"), None, p.pid)
        procs.append(p)
    for p in procs:
        assert p.wait(timeout=60) == 0  # 140 KB each: would block without a reader
    assert threading.active_count() == before + 1  # the pump thread only
    deadline = __import__("time").time() + 30
    while pump.streams and __import__("time").time() < deadline:
        __import__("time").sleep(0.05)
    assert pump.streams == 0  # every pipe reached EOF and was closed
    for k in range(12):
        lines = (tmp_path / f"w{k}.out").read_bytes().split(b"\n")
        assert lines[0].startswith(f"w{k} line 0 ".encode())
        assert lines[1999].startswith(f"w{k} line 1999 ".encode())
        assert lines[-1] == b"tail-no-newline"
    fwd = out.buffer.getvalue()
    assert fwd.count(b" line ") == 12 * 2000
    pump.stop()
