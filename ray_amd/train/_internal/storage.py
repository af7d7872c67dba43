"""Run storage on a pyarrow filesystem (reference: python/ray/train/_internal/storage.py
StorageContext).

``RunConfig(storage_path=..., storage_filesystem=...)`` selects where a run's
checkpoints and result files end up:

* a plain path and no filesystem: the local (or shared, e.g. NFS) filesystem, written
  in place — the common single-node case, no copies;
* ``storage_filesystem=<pyarrow.fs.FileSystem>``: ``storage_path`` is a path inside it;
* ``storage_path="<scheme>://..."``: the filesystem is resolved from the URI
  (``pyarrow.fs.FileSystem.from_uri``; ``file://`` resolves to the local case).

With a non-local filesystem, each run keeps a local staging directory for its driver
files (loggers, trainer state) under ``RAY_AMD_STORAGE`` (default ``~/ray_amd_results``),
workers upload reported checkpoints straight into
``<storage_path>/<run name>/checkpoint_<index>``, pruned checkpoints are deleted there,
and the staging files are uploaded when the run ends.
"""

from __future__ import annotations

import os


def _is_local(fs) -> bool:
    if fs is None:
        return True
    try:
        import pyarrow.fs as pafs
    except ImportError:  # pragma: no cover
        return False
    return isinstance(fs, pafs.LocalFileSystem)


def resolve(storage_path: str, storage_filesystem=None):
    """-> (filesystem or None for local, path within it)."""
    if storage_filesystem is not None:
        if _is_local(storage_filesystem):
            return None, os.path.abspath(os.path.expanduser(storage_path))
        return storage_filesystem, storage_path.rstrip("/")
    if "://" in storage_path:
        import pyarrow.fs as pafs

        fs, path = pafs.FileSystem.from_uri(storage_path)
        if _is_local(fs):
            return None, path
        return fs, path.rstrip("/")
    return None, os.path.abspath(os.path.expanduser(storage_path))


def join(*parts) -> str:
    return "/".join(p.rstrip("/") for p in parts if p)


def upload_dir(local_dir: str, fs, dst: str) -> None:
    import pyarrow.fs as pafs

    fs.create_dir(dst, recursive=True)
    pafs.copy_files(local_dir, dst, source_filesystem=pafs.LocalFileSystem(),
                    destination_filesystem=fs)


def download_dir(fs, src: str, local_dir: str) -> None:
    import pyarrow.fs as pafs

    os.makedirs(local_dir, exist_ok=True)
    pafs.copy_files(src, local_dir, source_filesystem=fs,
                    destination_filesystem=pafs.LocalFileSystem())


def delete_dir(fs, path: str) -> None:
    try:
        fs.delete_dir(path)
    except FileNotFoundError:
        pass


def list_dir(fs, path: str) -> list[str]:
    import pyarrow.fs as pafs

    try:
        infos = fs.get_file_info(pafs.FileSelector(path, allow_not_found=True))
    except FileNotFoundError:
        return []
    return [os.path.basename(i.path) for i in infos]


def read_text(fs, path: str) -> str | None:
    try:
        with fs.open_input_stream(path) as f:
            return f.read().decode()
    except (FileNotFoundError, OSError):
        return None


def write_text(fs, path: str, text: str) -> None:
    with fs.open_output_stream(path) as f:
        f.write(text.encode())
