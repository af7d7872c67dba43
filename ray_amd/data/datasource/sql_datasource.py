"""SQL reads and writes over DB-API 2 connections (reference: python/ray/data/datasource/
sql_datasource.py, sql_datasink.py): the query is sharded with LIMIT/OFFSET over its
COUNT(*) so parallel read tasks each pull one slice."""

from __future__ import annotations

from typing import Any, Callable, List

import numpy as np

from ray_amd.data import block as B
from ray_amd.data.datasource.datasink import Datasink
from ray_amd.data.datasource.datasource import Datasource, ReadTask

Connection = Any  # a DB-API 2 connection (reference: sql_datasource.Connection)


def _rows_to_block(cursor, rows) -> dict:
    cols = [d[0] for d in cursor.description]
    if not rows:
        return {c: np.array([]) for c in cols}
    return {c: B._col([r[i] for r in rows]) for i, c in enumerate(cols)}


class SQLDatasource(Datasource):
    def __init__(self, sql: str, connection_factory: Callable[[], Any], shard_keys=None):
        self.sql = sql.strip().rstrip(";")
        self.factory = connection_factory

    def _count(self) -> int:
        con = self.factory()
        try:
            cur = con.cursor()
            cur.execute(f"SELECT COUNT(*) FROM ({self.sql}) AS _ray_amd_q")
            return int(cur.fetchone()[0])
        finally:
            con.close()

    def get_read_tasks(self, parallelism: int) -> List[ReadTask]:
        sql, factory = self.sql, self.factory
        n = self._count()
        shards = max(1, min(parallelism, n)) if n else 1

        def task(limit, offset, whole):
            def read():
                con = factory()
                try:
                    cur = con.cursor()
                    if whole:
                        cur.execute(sql)
                    else:
                        cur.execute(f"SELECT * FROM ({sql}) AS _ray_amd_q "
                                    f"LIMIT {limit} OFFSET {offset}")
                    return _rows_to_block(cur, cur.fetchall())
                finally:
                    con.close()
            return ReadTask(read, {"num_rows": limit})

        if shards == 1:
            return [task(n, 0, True)]
        per = -(-n // shards)
        return [task(per, k * per, False) for k in range(shards) if k * per < n]


class SQLDatasink(Datasink):
    """``sql`` is an INSERT with one DB-API placeholder per column (block column order)."""

    def __init__(self, sql: str, connection_factory: Callable[[], Any]):
        self.sql = sql
        self.factory = connection_factory

    def write(self, blocks, ctx):
        con = self.factory()
        n = 0
        try:
            cur = con.cursor()
            for blk in blocks:
                rows = [tuple(B._py(v) for v in r.values()) for r in B.to_rows(blk)]
                if rows:
                    cur.executemany(self.sql, rows)
                    n += len(rows)
            con.commit()
        finally:
            con.close()
        return n

    def on_write_complete(self, write_results):
        return sum(write_results)


def read_sql(sql: str, connection_factory: Callable[[], Any], *, parallelism: int = -1,
             **kw):
    from ray_amd.data.read_api import _parallelism, read_datasource

    return read_datasource(SQLDatasource(sql, connection_factory),
                           parallelism=_parallelism(parallelism) if parallelism else 1)
