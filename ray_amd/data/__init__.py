"""ray_amd.data — streaming distributed datasets (reference: python/ray/data)."""

from ray_amd.data import aggregate  # noqa: F401,E402
from ray_amd.data.dataset import (ActorPoolStrategy, AggregateFn, Count, Dataset,  # noqa: F401
                                  GroupedData, Max, MaterializedDataset, Mean, Min, Std, Sum,
                                  TaskPoolStrategy)
from ray_amd.data.iterator import DataIterator  # noqa: F401
from ray_amd.data.block import Schema  # noqa: F401
from ray_amd.data.preprocessors import Preprocessor  # noqa: F401

DatasetIterator = DataIterator
NodeIdStr = str  # reference: data/_internal/execution/interfaces/common.py
from ray_amd.data.read_api import (from_arrow, from_arrow_refs, from_huggingface,  # noqa: F401
                                   from_items, from_numpy, from_numpy_refs, from_pandas,
                                   from_pandas_refs, from_torch, range, range_tensor,
                                   read_binary_files, read_csv, read_datasource, read_images,
                                   read_json, read_numpy, read_parquet, read_parquet_bulk,
                                   read_text, read_tfrecords, read_avro)
from ray_amd.data.integrations import (from_dask, from_mars, from_modin,  # noqa: F401
                                       from_spark, from_tf, read_bigquery,
                                       read_databricks_tables, read_mongo)
from ray_amd.data.datasource import (BlockBasedFileDatasink, Datasink,  # noqa: F401
                                     Datasource, ReadTask, RowBasedFileDatasink,
                                     FileBasedDatasource, read_sql, read_webdataset)
from ray_amd.data.random_access_dataset import RandomAccessDataset  # noqa: F401
from ray_amd.data import preprocessors  # noqa: F401
from ray_amd.data._executor import ExecutionOptions, ExecutionResources  # noqa: F401


from ray_amd.data.context import DataContext, DatasetContext  # noqa: E402,F401


def set_progress_bars(enabled: bool) -> bool:
    """Enable/disable execution progress output; returns the previous setting."""
    ctx = DataContext.get_current()
    old = getattr(ctx, "enable_progress_bars", True)
    ctx.enable_progress_bars = bool(enabled)
    return old
