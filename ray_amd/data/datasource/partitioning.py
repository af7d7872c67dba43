"""Path-based partitioning (reference: python/ray/data/datasource/partitioning.py).

``Partitioning("hive")`` reads ``key=value`` directory segments; ``Partitioning("dirs",
field_names=[...])`` names the last directory segments. ``PathPartitionParser`` turns a
file path into its partition values (typed with ``field_types``); ``PathPartitionFilter``
keeps the paths whose values satisfy a predicate — file-based reads apply it before any
file is opened, and add the values as columns of the rows read."""

from __future__ import annotations

import os
from dataclasses import dataclass
from enum import Enum
from typing import Any, Callable, Dict, List, Optional


class PartitionStyle(str, Enum):
    HIVE = "hive"
    DIRECTORY = "dirs"


@dataclass
class Partitioning:
    style: PartitionStyle = PartitionStyle.HIVE
    base_dir: Optional[str] = None
    field_names: Optional[List[str]] = None
    field_types: Optional[Dict[str, type]] = None
    filesystem: Any = None

    def __post_init__(self):
        self.style = PartitionStyle(self.style)
        if self.style == PartitionStyle.DIRECTORY and not self.field_names:
            raise ValueError("directory partitioning needs field_names")
        self.field_types = dict(self.field_types or {})

    @property
    def normalized_base_dir(self) -> str:
        return (os.path.abspath(self.base_dir).rstrip(os.sep) + os.sep) if self.base_dir \
            else ""


def _cast(values: Dict[str, str], types: Dict[str, type]) -> Dict[str, Any]:
    out = {}
    for k, v in values.items():
        t = types.get(k)
        if t is bool:
            out[k] = v.lower() in ("true", "1")
        else:
            out[k] = t(v) if t is not None else v
    return out


class PathPartitionParser:
    def __init__(self, partitioning: Partitioning):
        self._scheme = partitioning

    @staticmethod
    def of(style: PartitionStyle = PartitionStyle.HIVE, base_dir: Optional[str] = None,
           field_names: Optional[List[str]] = None,
           field_types: Optional[Dict[str, type]] = None,
           filesystem=None) -> "PathPartitionParser":
        return PathPartitionParser(Partitioning(style, base_dir, field_names, field_types,
                                                filesystem))

    @property
    def scheme(self) -> Partitioning:
        return self._scheme

    def _dir_segments(self, path: str, base: Optional[str] = None) -> List[str]:
        base = self._scheme.normalized_base_dir or base
        d = os.path.dirname(os.path.abspath(path) if "://" not in path else path)
        if base:
            b = base.rstrip(os.sep)
            if not (d == b or d.startswith(b + os.sep)):
                return []
            d = d[len(b):]
        return [s for s in d.split(os.sep) if s]

    def __call__(self, path: str, base: Optional[str] = None) -> Dict[str, Any]:
        """Partition values of ``path`` (``base``: the read's root directory, when the
        scheme names none)."""
        segs = self._dir_segments(path, base)
        if self._scheme.style == PartitionStyle.HIVE:
            vals = {}
            for s in segs:
                k, sep, v = s.partition("=")
                if sep and k:
                    vals[k] = v
        else:
            names = self._scheme.field_names
            if len(segs) < len(names):
                return {}
            vals = dict(zip(names, segs[len(segs) - len(names):]))
        return _cast(vals, self._scheme.field_types)


class PathPartitionFilter:
    """Callable over a list of paths: the ones whose partition values pass ``filter_fn``
    (paths without partition values are kept, as in the reference)."""

    @staticmethod
    def of(filter_fn: Callable[[Dict[str, Any]], bool],
           style: PartitionStyle = PartitionStyle.HIVE, base_dir: Optional[str] = None,
           field_names: Optional[List[str]] = None,
           field_types: Optional[Dict[str, type]] = None,
           filesystem=None) -> "PathPartitionFilter":
        return PathPartitionFilter(PathPartitionParser.of(style, base_dir, field_names,
                                                          field_types, filesystem), filter_fn)

    def __init__(self, path_partition_parser: PathPartitionParser,
                 filter_fn: Callable[[Dict[str, Any]], bool]):
        self._parser = path_partition_parser
        self._filter_fn = filter_fn

    @property
    def parser(self) -> PathPartitionParser:
        return self._parser

    def __call__(self, paths: List[str], base: Optional[str] = None) -> List[str]:
        out = []
        for p in paths:
            vals = self._parser(p, base)
            if not vals or self._filter_fn(vals):
                out.append(p)
        return out
