"""Worker log deduplication on the driver terminal (modelled on
python/ray/tests/test_log_dedup.py)."""

import io
import os
import subprocess
import sys
import textwrap
import time

from ray_amd._private.log_dedup import LogDeduplicator, canonicalise

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_canonicalise_drops_words_with_numbers():
    assert canonicalise("step 12 loss=0.5 done") == "step done"
    assert canonicalise("worker 0xdeadbeef ready") == "worker ready"


def test_dedup_window_and_repeat_summary():
    out = io.StringIO()
    d = LogDeduplicator(window_s=0.3, background=False)
    first = d.feed(b"hello from pid 1\n", 1, out)
    assert first == [b"hello from pid 1\n"]
    assert d.feed(b"hello from pid 2\n", 2, out) == []
    assert d.feed(b"hello from pid 3\n", 3, out) == []
    assert d.feed(b"something else\n", 1, out) == [b"something else\n"]
    # one process repeating itself is printed, not counted
    assert d.feed(b"loop 1\n", 7, out) == [b"loop 1\n"]
    assert d.feed(b"loop 2\n", 7, out) == [b"loop 2\n"]
    time.sleep(0.4)
    ready = d.flush()
    assert ready == [(out, "hello from pid 3 [repeated 2x across cluster]\n")]
    # the window closed: the next one prints again
    assert d.feed(b"hello from pid 4\n", 4, out) == [b"hello from pid 4\n"]


def test_disable_allow_and_skip():
    out = io.StringIO()
    off = LogDeduplicator(enabled=False)
    assert off.feed(b"x\n", 1, out) == [b"x\n"] and off.feed(b"x\n", 2, out) == [b"x\n"]
    d = LogDeduplicator(allow_re="KEEP", skip_re="DROP")
    assert d.feed(b"KEEP me\n", 1, out) == [b"KEEP me\n"]
    assert d.feed(b"KEEP me\n", 2, out) == [b"KEEP me\n"]
    assert d.feed(b"DROP me\n", 1, out) == []


def test_driver_sees_repeats_collapsed():
    code = textwrap.dedent('''
        import sys, time
        sys.path.insert(0, %r)
        import ray_amd as ray
        ray.init(num_cpus=4)

        @ray.remote
        class Noisy:
            def say(self, i):
                print("dedup-me task output", flush=True)
                return i

        actors = [Noisy.remote() for _ in range(4)]  # four processes
        ray.get([a.say.remote(i) for i, a in enumerate(actors)])
        ray.get([a.say.remote(i) for i, a in enumerate(actors)])
        time.sleep(2.5)
        ray.shutdown()
    ''' % REPO)
    env = dict(os.environ, RAY_DEDUP_LOGS_AGG_WINDOW_S="1")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                       timeout=120, env=env)
    lines = [ln for ln in r.stdout.splitlines() if "dedup-me" in ln]
    assert sum("repeated" not in ln for ln in lines) >= 1
    assert any("[repeated" in ln and "across cluster]" in ln for ln in lines), r.stdout
    total = sum(int(ln.split("[repeated ")[1].split("x")[0]) if "[repeated" in ln else 1
                for ln in lines)
    assert total == 8
