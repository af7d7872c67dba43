"""The built-in file formats as ``FileBasedDatasource`` subclasses (reference:
python/ray/data/datasource/{csv,json,parquet,numpy,text,binary,image,tfrecords,avro,
webdataset}_datasource.py). ``read_api.read_*`` construct these; each is also usable
directly with ``read_datasource``."""

from __future__ import annotations

import io
from typing import Any, Dict, List, Optional

import numpy as np

from ray_amd.data.datasource.file_based_datasource import FileBasedDatasource


class CSVDatasource(FileBasedDatasource):
    _FILE_EXTENSIONS = ["csv", "csv.gz"]

    def __init__(self, paths, arrow_csv_args: Optional[Dict[str, Any]] = None, **kw):
        super().__init__(paths, **kw)
        self.arrow_csv_args = dict(arrow_csv_args or {})

    def _read_stream(self, f, path):
        import pyarrow.csv as pc

        a = dict(self.arrow_csv_args)
        opts = {k: a.pop(k) for k in ("read_options", "parse_options", "convert_options")
                if k in a}
        yield pc.read_csv(f, **opts)


class JSONDatasource(FileBasedDatasource):
    _FILE_EXTENSIONS = ["json", "jsonl", "json.gz", "jsonl.gz"]

    def __init__(self, paths, lines: Optional[bool] = None, **kw):
        super().__init__(paths, **kw)
        self.lines = lines

    def _read_stream(self, f, path):
        import pandas as pd

        data = f.read()
        if self.lines is not False:
            try:
                yield pd.read_json(io.BytesIO(data), lines=True)
                return
            except ValueError:
                if self.lines:
                    raise
        yield pd.read_json(io.BytesIO(data))


class ParquetDatasource(FileBasedDatasource):
    _FILE_EXTENSIONS = ["parquet"]

    def __init__(self, paths, columns: Optional[List[str]] = None, **kw):
        kw.pop("dataset_kwargs", None)
        kw.pop("tensor_column_schema", None)
        super().__init__(paths, **kw)
        self.columns = columns

    def _read_file(self, path):
        import pyarrow.parquet as pq

        # tensor extension columns (ray.data.arrow_tensor) must be registered in the
        # reading process, or they load as plain lists
        from ray_amd.data.extensions import tensor_extension  # noqa: F401

        return pq.read_table(path, columns=self.columns, partitioning=None,
                             filesystem=self._filesystem)


ParquetBaseDatasource = ParquetDatasource


class NumpyDatasource(FileBasedDatasource):
    _FILE_EXTENSIONS = ["npy"]

    def _read_stream(self, f, path):
        yield {"data": np.load(io.BytesIO(f.read()), allow_pickle=False)}


class TextDatasource(FileBasedDatasource):
    def __init__(self, paths, drop_empty_lines: bool = True, encoding: str = "utf-8", **kw):
        super().__init__(paths, **kw)
        self.drop_empty_lines = drop_empty_lines
        self.encoding = encoding

    def _read_stream(self, f, path):
        lines = f.read().decode(self.encoding).split("\n")
        if lines and lines[-1] == "":
            lines = lines[:-1]
        if self.drop_empty_lines:
            lines = [ln for ln in lines if ln.strip()]
        yield {"text": np.array(lines, dtype=object)}


class BinaryDatasource(FileBasedDatasource):
    _COLUMN_NAME = "bytes"

    def _read_stream(self, f, path):
        b = np.empty(1, dtype=object)
        b[0] = f.read()
        yield {self._COLUMN_NAME: b}


class ImageDatasource(FileBasedDatasource):
    """Image files (png/jpg/bmp/gif/webp/tiff via PIL, or .npy HWC arrays) as rows with an
    ``image`` HWC uint8 array; ``size=(h, w)`` resizes, ``mode`` converts (e.g. "RGB")."""

    _FILE_EXTENSIONS = ["png", "jpg", "jpeg", "bmp", "gif", "webp", "tif", "tiff", "npy"]

    def __init__(self, paths, size=None, mode=None, **kw):
        super().__init__(paths, **kw)
        self.size, self.mode = size, mode

    def _read_stream(self, f, path):
        data = f.read()
        if path.endswith(".npy"):
            img = np.load(io.BytesIO(data), allow_pickle=False)
        else:
            from PIL import Image

            im = Image.open(io.BytesIO(data))
            if self.mode is not None:
                im = im.convert(self.mode)
            if self.size is not None:
                im = im.resize((self.size[1], self.size[0]))
            img = np.asarray(im)
        yield {"image": img[None]}


class TFRecordDatasource(FileBasedDatasource):
    """TFRecord files of tf.train.Example protos (data/tfrecords.py); ``verify`` checks
    every record's CRC32C."""

    _FILE_EXTENSIONS = ["tfrecords", "tfrecord", "gz"]

    def __init__(self, paths, tf_schema=None, verify: bool = True, compression=None, **kw):
        if tf_schema is not None:
            raise NotImplementedError("tf_schema needs tensorflow_metadata (not installed)")
        super().__init__(paths, **kw)
        self.verify = verify
        self.compression = compression or self._open_stream_args.get("compression")

    def _read_file(self, path):
        from ray_amd.data.tfrecords import read_file

        return read_file(path, self.verify, self.compression)


class AvroDatasource(FileBasedDatasource):
    """Avro object container files (data/avro.py): a column per top-level record field."""

    _FILE_EXTENSIONS = ["avro"]

    def _read_file(self, path):
        from ray_amd.data.avro import read_file

        return read_file(path)


class WebDatasetDatasource(FileBasedDatasource):
    _FILE_EXTENSIONS = ["tar", "tar.gz", "tgz"]

    def __init__(self, paths, decoder: bool = True, suffixes=None, **kw):
        super().__init__(paths, **kw)
        self.decoder, self.suffixes = decoder, suffixes

    def _read_file(self, path):
        from ray_amd.data.datasource.webdataset_datasource import _read_tar

        return _read_tar(path, self.decoder, self.suffixes)
