"""Path helpers of file-based reads (reference: python/ray/data/datasource/path_util.py)."""

from __future__ import annotations

import glob
import os
from typing import List, Optional, Tuple


def _has_file_extension(path: str, extensions: Optional[List[str]]) -> bool:
    if not extensions:
        return True
    p = path.lower()
    return any(p.endswith(e.lower() if e.startswith(".") else "." + e.lower())
               for e in extensions)


def _is_local_scheme(paths) -> bool:
    paths = [paths] if isinstance(paths, str) else paths
    return all(p.startswith("local://") for p in paths)


def _strip_scheme(path: str) -> str:
    for s in ("local://", "file://"):
        if path.startswith(s):
            return path[len(s):]
    return path


def _resolve_paths_and_filesystem(paths, filesystem=None) -> Tuple[List[str], object]:
    """(paths, pyarrow filesystem or None for the local one). URIs with a scheme resolve
    through ``pyarrow.fs.FileSystem.from_uri``."""
    if isinstance(paths, str):
        paths = [paths]
    out = []
    for p in paths:
        p = _strip_scheme(os.fspath(p))
        if filesystem is None and "://" in p:
            import pyarrow.fs as pafs

            filesystem, p = pafs.FileSystem.from_uri(p)
        out.append(p if filesystem is not None else os.path.expanduser(p))
    return out, filesystem


def _expand_local(p: str) -> List[str]:
    if os.path.isdir(p):
        files = []
        for root, dirs, names in os.walk(p):
            dirs.sort()
            for n in sorted(names):
                if not n.startswith(".") and not n.startswith("_"):
                    files.append(os.path.join(root, n))
        return files
    if any(c in p for c in "*?["):
        return sorted(glob.glob(p))
    return [p]
