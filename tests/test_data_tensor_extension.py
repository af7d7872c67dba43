"""Tensor extension types in the reference's on-disk form (data/extensions): Arrow arrays
round-trip N-d tensors, Parquet files carrying ``ray.data.arrow_tensor`` columns read back
as tensor columns, and the pandas TensorArray column behaves as a column of ndarrays."""
import numpy as np
import pandas as pd
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

import ray_amd as ray
import ray_amd.data as rd
from ray_amd.data.extensions import (ArrowTensorArray, ArrowTensorType,
                                     ArrowVariableShapedTensorArray, TensorArray,
                                     TensorDtype, column_needs_tensor_extension)


def test_arrow_tensor_roundtrip_and_metadata():
    x = np.arange(2 * 3 * 4, dtype=np.float32).reshape(2, 3, 4)
    a = ArrowTensorArray.from_numpy(x)
    assert isinstance(a.type, ArrowTensorType) and a.type.shape == (3, 4)
    assert a.type.extension_name == "ray.data.arrow_tensor"
    assert a.type.__arrow_ext_serialize__() == b"[3, 4]"
    assert np.array_equal(a.to_numpy(), x)
    v = ArrowTensorArray.from_numpy([np.ones((2, 2)), np.zeros((3, 1))])
    assert isinstance(v, ArrowVariableShapedTensorArray)
    got = v.to_numpy()
    assert got[0].shape == (2, 2) and got[1].shape == (3, 1)


def test_parquet_tensor_column_reads_as_tensor(tmp_path):
    x = np.random.default_rng(0).random((6, 2, 3)).astype(np.float32)
    t = pa.table({"id": pa.array(range(6)), "img": ArrowTensorArray.from_numpy(x)})
    pq.write_table(t, tmp_path / "t.parquet")
    back = pq.read_table(tmp_path / "t.parquet")
    assert isinstance(back.schema.field("img").type, ArrowTensorType)
    ray.init(num_cpus=2)
    try:
        b = next(iter(rd.read_parquet(str(tmp_path)).iter_batches(batch_size=6)))
        assert b["img"].shape == (6, 2, 3) and np.allclose(b["img"], x)
    finally:
        ray.shutdown()


def test_pandas_tensor_array():
    x = np.arange(12).reshape(4, 3)
    s = pd.Series(TensorArray(x))
    assert isinstance(s.dtype, TensorDtype) and s.dtype.element_shape == (3,)
    assert np.array_equal(np.asarray(s.iloc[2]), [6, 7, 8])
    assert np.array_equal(s.iloc[1:3].values.to_numpy(), x[1:3])
    df = pd.DataFrame({"t": TensorArray(x), "k": [0, 1, 0, 1]})
    assert np.array_equal(df[df.k == 1]["t"].values.to_numpy(), x[[1, 3]])
    assert column_needs_tensor_extension(pd.Series([np.zeros(2), np.ones(2)]))
    tbl = pa.Table.from_pandas(df)
    assert isinstance(tbl.schema.field("t").type, ArrowTensorType)
    with pytest.raises(TypeError):
        TensorDtype.construct_from_string("nope")
