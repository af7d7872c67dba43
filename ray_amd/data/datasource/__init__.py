"""``ray_amd.data.datasource`` (reference: python/ray/data/datasource/__init__.py):
custom sources and sinks, the file-based reader framework, partitioning, and the
built-in formats' datasources / datasinks."""

from ray_amd.data.datasource.block_path_provider import (  # noqa: F401
    BlockWritePathProvider, DefaultBlockWritePathProvider)
from ray_amd.data.datasource.datasink import (Datasink, DummyOutputDatasink,  # noqa: F401
                                              _sink_write, write_datasink)
from ray_amd.data.datasource.datasource import Datasource, ReadTask, Reader  # noqa: F401
from ray_amd.data.datasource.file_based_datasource import (  # noqa: F401
    FileBasedDatasource, FileExtensionFilter)
from ray_amd.data.datasource.file_datasink import (  # noqa: F401
    BlockBasedFileDatasink, RowBasedFileDatasink, _CSVDatasink, _ImageDatasink,
    _JSONDatasink, _NumpyDatasink, _ParquetDatasink, _TFRecordDatasink, _WebDatasetDatasink)
from ray_amd.data.datasource.file_meta_provider import (  # noqa: F401
    BaseFileMetadataProvider, DefaultFileMetadataProvider, DefaultParquetMetadataProvider,
    FastFileMetadataProvider, FileMetadataProvider, ParquetMetadataProvider)
from ray_amd.data.datasource.filename_provider import FilenameProvider  # noqa: F401
from ray_amd.data.datasource.formats import (  # noqa: F401
    AvroDatasource, BinaryDatasource, CSVDatasource, ImageDatasource, JSONDatasource,
    NumpyDatasource, ParquetBaseDatasource, ParquetDatasource, TextDatasource,
    TFRecordDatasource, WebDatasetDatasource)
from ray_amd.data.datasource.image_datasink import _write_images_block  # noqa: F401
from ray_amd.data.datasource.other_sources import (  # noqa: F401
    BigQueryDatasource, DatabricksUCDatasource, HuggingFaceDatasource, MongoDatasource,
    RandomIntRowDatasource, RangeDatasource, TorchDatasource)
from ray_amd.data.datasource.partitioning import (  # noqa: F401
    Partitioning, PartitionStyle, PathPartitionFilter, PathPartitionParser)
from ray_amd.data.datasource.sql_datasource import (  # noqa: F401
    Connection, SQLDatasink, SQLDatasource, read_sql)
from ray_amd.data.datasource.webdataset_datasource import (  # noqa: F401
    _write_tar, read_webdataset)

_SQLDatasink = SQLDatasink


class _MongoDatasink(Datasink):
    def __init__(self, uri: str, database: str, collection: str):
        self.uri, self.database, self.collection = uri, database, collection

    def write(self, blocks, ctx):
        from ray_amd.data import block as B
        from ray_amd.data.integrations import _need

        pymongo = _need("pymongo", "pymongo", "Dataset.write_mongo")
        coll = pymongo.MongoClient(self.uri)[self.database][self.collection]
        n = 0
        for blk in blocks:
            rows = [{k: B._py(v) for k, v in r.items()} for r in B.to_rows(blk)]
            if rows:
                coll.insert_many(rows)
                n += len(rows)
        return n


class _BigQueryDatasink(Datasink):
    def __init__(self, project_id: str, dataset: str, **kw):
        from ray_amd.data.integrations import _need

        _need("google.cloud.bigquery", "google-cloud-bigquery", "Dataset.write_bigquery")


class _S3FileSystemWrapper:
    """Pickle wrapper of a pyarrow S3FileSystem (the reference's; pyarrow filesystems
    pickle natively in the pyarrow of this image, so this only holds the object)."""

    def __init__(self, fs):
        self._fs = fs

    def unwrap(self):
        return self._fs


__all__ = [n for n in dir() if not n.startswith("__") and n not in ("annotations",)]
