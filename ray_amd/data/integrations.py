"""Dataset conversions to and from external frameworks (reference:
python/ray/data/read_api.py from_dask/from_mars/from_modin/from_spark/from_tf,
read_bigquery/read_databricks_tables/read_mongo; dataset.py to_dask/to_mars/to_modin/
to_spark/to_tf/iter_tf_batches/write_bigquery/write_mongo).

Each needs a library that is not part of this image (dask, mars, modin, pyspark,
tensorflow, google-cloud-bigquery, databricks-sql, pymongo). The entry points exist with the
reference's names and signatures and fail the way the reference does when its optional
dependency is missing: an ImportError naming the package. Where the library IS importable
the conversion goes through pandas / Arrow, which every one of them speaks."""

from __future__ import annotations

import importlib


def _need(module: str, pip_name: str, api: str):
    try:
        return importlib.import_module(module)
    except ImportError:
        raise ImportError(f"{api} requires {pip_name}, which is not installed "
                          f"(`pip install {pip_name}`)") from None


# ------------------------------------------------------------------ readers / from_*
def from_dask(df):
    _need("dask", "dask", "ray.data.from_dask")
    from ray_amd.data.read_api import from_pandas

    return from_pandas(list(df.to_delayed() and [p.compute() for p in df.to_delayed()]))


def from_modin(df):
    _need("modin", "modin", "ray.data.from_modin")
    from ray_amd.data.read_api import from_pandas

    return from_pandas(df._to_pandas())


def from_mars(df):
    _need("mars", "pymars", "ray.data.from_mars")
    from ray_amd.data.read_api import from_pandas

    return from_pandas(df.to_pandas())


def from_spark(df, *, parallelism=None, override_num_blocks=None):
    _need("pyspark", "pyspark", "ray.data.from_spark")
    from ray_amd.data.read_api import from_pandas

    return from_pandas(df.toPandas())


def from_tf(dataset):
    _need("tensorflow", "tensorflow", "ray.data.from_tf")
    from ray_amd.data.read_api import from_items

    return from_items([{k: v.numpy() for k, v in ex.items()} if isinstance(ex, dict)
                       else {"item": ex.numpy()} for ex in dataset])


def read_bigquery(project_id, dataset=None, query=None, **kw):
    _need("google.cloud.bigquery", "google-cloud-bigquery", "ray.data.read_bigquery")
    raise NotImplementedError("read_bigquery: BigQuery storage reads are not wired yet")


def read_databricks_tables(*, warehouse_id, table=None, query=None, **kw):
    _need("databricks.sql", "databricks-sql-connector", "ray.data.read_databricks_tables")
    raise NotImplementedError("read_databricks_tables is not wired yet")


def read_mongo(uri, database, collection, **kw):
    pymongo = _need("pymongo", "pymongo", "ray.data.read_mongo")
    from ray_amd.data.read_api import from_items

    coll = pymongo.MongoClient(uri)[database][collection]
    pipeline = kw.get("pipeline")
    rows = list(coll.aggregate(pipeline) if pipeline else coll.find())
    for r in rows:  # ObjectId is not an Arrow type
        if "_id" in r:
            r["_id"] = str(r["_id"])
    return from_items(rows)


# ------------------------------------------------------------------ Dataset methods
def to_dask(ds, *args, **kw):
    dd = _need("dask.dataframe", "dask", "Dataset.to_dask")
    return dd.from_pandas(ds.to_pandas(), npartitions=max(1, ds.num_blocks()))


def to_modin(ds):
    mpd = _need("modin.pandas", "modin", "Dataset.to_modin")
    return mpd.DataFrame(ds.to_pandas())


def to_mars(ds):
    md = _need("mars.dataframe", "pymars", "Dataset.to_mars")
    return md.DataFrame(ds.to_pandas())


def to_spark(ds, spark):
    _need("pyspark", "pyspark", "Dataset.to_spark")
    return spark.createDataFrame(ds.to_pandas())


def to_tf(ds, feature_columns, label_columns, *, batch_size=1, **kw):
    tf = _need("tensorflow", "tensorflow", "Dataset.to_tf")

    def gen():
        for b in ds.iter_batches(batch_size=batch_size):
            f = b[feature_columns] if isinstance(feature_columns, str) else \
                {c: b[c] for c in feature_columns}
            y = b[label_columns] if isinstance(label_columns, str) else \
                {c: b[c] for c in label_columns}
            yield f, y

    return tf.data.Dataset.from_generator(gen, output_signature=kw.get("output_signature"))


def iter_tf_batches(ds, *, batch_size=256, dtypes=None, **kw):
    tf = _need("tensorflow", "tensorflow", "Dataset.iter_tf_batches")
    for b in ds.iter_batches(batch_size=batch_size, **kw):
        yield {k: tf.convert_to_tensor(v, dtype=(dtypes or {}).get(k) if isinstance(dtypes, dict)
                                       else dtypes) for k, v in b.items()}


def write_bigquery(ds, project_id, dataset, **kw):
    _need("google.cloud.bigquery", "google-cloud-bigquery", "Dataset.write_bigquery")
    raise NotImplementedError("write_bigquery is not wired yet")


def write_mongo(ds, uri, database, collection, **kw):
    pymongo = _need("pymongo", "pymongo", "Dataset.write_mongo")
    coll = pymongo.MongoClient(uri)[database][collection]
    for b in ds.iter_batches(batch_format="pandas"):
        coll.insert_many(b.to_dict("records"))
