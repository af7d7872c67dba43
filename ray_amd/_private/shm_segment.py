"""Shared-memory segments that cannot outlive the processes using them.

Reference: plasma maps its arena and unlinks the backing file immediately "so we do not
leave traces in the system" (src/ray/object_manager/plasma/dlmalloc.cc:143,162-165), and
hands the fd to clients over the store socket (SCM_RIGHTS).

Here every node's object store and every compiled-graph channel is an anonymous
``memfd`` created by the process that owns it. Other local processes open it through
``/proc/<owner pid>/fd/<fd>`` — a path that exists exactly as long as the owner holds the
fd — so nothing is ever named in ``/dev/shm``. The kernel frees the pages when the last
process that holds the fd or maps the segment exits, whatever way it exits (SIGKILL of a
node agent by ``Cluster.shutdown``, a crashed raylet, an OOM kill).

``RAY_AMD_SHM_MEMFD=0`` restores named ``/dev/shm`` files (for tools that want to see
them); ``sweep_dead`` then removes the files of sessions whose creating process is gone,
which every ``ray_amd.init`` runs.
"""

from __future__ import annotations

import os
import re

_MEMFD = os.environ.get("RAY_AMD_SHM_MEMFD", "1") != "0" and hasattr(os, "memfd_create")


def memfd_enabled() -> bool:
    return _MEMFD


def create(path: str) -> tuple[str, int | None]:
    """Returns ``(open_path, fd)``: the path other local processes open the segment by,
    and the fd the owner keeps open for the segment's lifetime (None for a named file,
    which the owner unlinks in ``release``). The caller sizes and maps it (``_core``)."""
    if not _MEMFD:
        return path, None
    fd = os.memfd_create(os.path.basename(path)[:200] or "ray_amd", os.MFD_CLOEXEC)
    return f"/proc/{os.getpid()}/fd/{fd}", fd


def release(path: str, fd: int | None) -> None:
    """End the owner's reference: close the memfd (mappings elsewhere stay valid until
    those processes unmap) or unlink the named file."""
    try:
        if fd is not None:
            os.close(fd)
        elif path and not path.startswith("/proc/"):
            os.unlink(path)
    except OSError:
        pass


def is_anonymous(path: str) -> bool:
    return path.startswith("/proc/")


_PID_RE = (re.compile(r"^ray_amd_session_[0-9-]+_[0-9-]+_(\d+)_"), re.compile(r"^ramd_ch_(\d+)_"))


def _alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    return True


def sweep_dead(shm_dir: str = "/dev/shm") -> list[str]:
    """Remove named segments (from ``RAY_AMD_SHM_MEMFD=0`` runs or older versions) whose
    creating process — the pid in the session / channel name — no longer exists. A live
    pid (possibly reused) keeps its files: the sweep only ever errs on the side of leaving
    a file."""
    removed = []
    try:
        names = os.listdir(shm_dir)
    except OSError:
        return removed
    for n in names:
        for rx in _PID_RE:
            m = rx.match(n)
            if m is None:
                continue
            if not _alive(int(m.group(1))):
                try:
                    os.unlink(os.path.join(shm_dir, n))
                    removed.append(n)
                except OSError:
                    pass
            break
    return removed
