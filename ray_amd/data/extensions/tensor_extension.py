"""Tensor columns as Arrow / pandas extension types (reference API:
python/ray/data/extensions/__init__.py over air/util/tensor_extensions/{arrow,pandas}.py).

The Arrow types use the reference's on-disk form, so Parquet / Feather files holding tensor
columns written by Ray read here as tensors, and files written with these types read there:

* ``ArrowTensorType(shape, dtype)``: extension name ``ray.data.arrow_tensor``, storage
  ``list<dtype>`` with one flattened tensor per row, metadata = the JSON element shape;
* ``ArrowVariableShapedTensorType(dtype, ndim)``: ``ray.data.arrow_variable_shaped_tensor``,
  storage ``struct<data: list<dtype>, shape: list<int64>>``, metadata = the JSON ndim.

ray_amd's own blocks keep fixed-shape tensor columns as nested fixed-size lists
(data/block.py); ``data.block`` turns either extension type into an N-d numpy column on
read. ``TensorDtype`` / ``TensorArray`` are the pandas side: a column of equally shaped
ndarrays in a DataFrame, backed by one (N, *shape) ndarray.
"""

from __future__ import annotations

import json
import numbers

import numpy as np
import pandas as pd
import pyarrow as pa


# ------------------------------------------------------------------------------ Arrow
class ArrowTensorType(pa.ExtensionType):
    def __init__(self, shape, dtype):
        self._shape = tuple(int(s) for s in shape)
        super().__init__(pa.list_(dtype), "ray.data.arrow_tensor")

    @property
    def shape(self):
        return self._shape

    @property
    def scalar_type(self):
        return self.storage_type.value_type

    def __arrow_ext_serialize__(self):
        return json.dumps(list(self._shape)).encode()

    @classmethod
    def __arrow_ext_deserialize__(cls, storage_type, serialized):
        return cls(tuple(json.loads(serialized)), storage_type.value_type)

    def __arrow_ext_class__(self):
        return ArrowTensorArray

    def __reduce__(self):
        return self.__arrow_ext_deserialize__, (self.storage_type,
                                                self.__arrow_ext_serialize__())

    def to_pandas_dtype(self):
        return TensorDtype(self._shape, self.scalar_type.to_pandas_dtype())


class ArrowTensorArray(pa.ExtensionArray):
    @classmethod
    def from_numpy(cls, arr, column_name=None):
        """(N, *shape) ndarray, or a sequence of ndarrays (variable shapes give an
        ``ArrowVariableShapedTensorArray``)."""
        if not isinstance(arr, np.ndarray) or arr.dtype == object:
            arrs = [np.asarray(a) for a in arr]
            if arrs and all(a.shape == arrs[0].shape for a in arrs):
                arr = np.stack(arrs)
            else:
                return ArrowVariableShapedTensorArray.from_numpy(arrs)
        arr = np.ascontiguousarray(arr)
        n = arr.shape[0]
        shape = arr.shape[1:]
        flat = pa.array(arr.reshape(-1))
        size = int(np.prod(shape)) if shape else 1
        offsets = pa.array(np.arange(0, (n + 1) * size, size, dtype=np.int32))
        storage = pa.ListArray.from_arrays(offsets, flat)
        return pa.ExtensionArray.from_storage(ArrowTensorType(shape, flat.type), storage)

    def to_numpy(self, zero_copy_only: bool = False):
        shape = self.type.shape
        flat = self.storage.flatten().to_numpy(zero_copy_only=False)
        return flat.reshape((len(self),) + tuple(shape))

    def to_pylist(self):
        return list(self.to_numpy())


class ArrowVariableShapedTensorType(pa.ExtensionType):
    def __init__(self, dtype, ndim: int):
        self._ndim = int(ndim)
        super().__init__(pa.struct([("data", pa.list_(dtype)),
                                    ("shape", pa.list_(pa.int64()))]),
                         "ray.data.arrow_variable_shaped_tensor")

    @property
    def ndim(self):
        return self._ndim

    @property
    def scalar_type(self):
        return self.storage_type[self.storage_type.get_field_index("data")].type.value_type

    def __arrow_ext_serialize__(self):
        return json.dumps(self._ndim).encode()

    @classmethod
    def __arrow_ext_deserialize__(cls, storage_type, serialized):
        return cls(storage_type["data"].type.value_type, json.loads(serialized))

    def __arrow_ext_class__(self):
        return ArrowVariableShapedTensorArray

    def __reduce__(self):
        return self.__arrow_ext_deserialize__, (self.storage_type,
                                                self.__arrow_ext_serialize__())


class ArrowVariableShapedTensorArray(pa.ExtensionArray):
    @classmethod
    def from_numpy(cls, arrs):
        arrs = [np.ascontiguousarray(a) for a in arrs]
        if not arrs:
            raise ValueError("no tensors")
        ndim = arrs[0].ndim
        if any(a.ndim != ndim for a in arrs):
            raise ValueError("variable-shaped tensors must share their number of dimensions")
        dtype = np.result_type(*arrs)
        flat = pa.array(np.concatenate([a.astype(dtype, copy=False).reshape(-1)
                                        for a in arrs]))
        sizes = np.array([a.size for a in arrs], np.int64)
        offsets = pa.array(np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32))
        data = pa.ListArray.from_arrays(offsets, flat)
        shapes = pa.array([list(a.shape) for a in arrs], pa.list_(pa.int64()))
        storage = pa.StructArray.from_arrays([data, shapes], ["data", "shape"])
        return pa.ExtensionArray.from_storage(
            ArrowVariableShapedTensorType(flat.type, ndim), storage)

    def to_numpy(self, zero_copy_only: bool = False):
        data = self.storage.field("data")
        shapes = self.storage.field("shape").to_pylist()
        out = np.empty(len(self), dtype=object)
        for i, shp in enumerate(shapes):
            out[i] = data[i].values.to_numpy(zero_copy_only=False).reshape(shp)
        return out

    def to_pylist(self):
        return list(self.to_numpy())


for _t in (ArrowTensorType((0,), pa.int64()), ArrowVariableShapedTensorType(pa.int64(), 0)):
    try:
        pa.register_extension_type(_t)
    except pa.ArrowKeyError:  # registered by an earlier import (or by real Ray)
        pass


# ------------------------------------------------------------------------------ pandas
@pd.api.extensions.register_extension_dtype
class TensorDtype(pd.api.extensions.ExtensionDtype):
    """dtype of a pandas column whose cells are ndarrays of one shape and element type."""

    name = "TensorDtype"
    kind = "O"
    na_value = np.nan

    def __init__(self, shape=(), dtype=np.float64):
        self._shape = tuple(shape)
        self._dtype = np.dtype(dtype)

    @property
    def type(self):
        return TensorArrayElement

    @property
    def element_shape(self):
        return self._shape

    @property
    def element_dtype(self):
        return self._dtype

    @classmethod
    def construct_array_type(cls):
        return TensorArray

    @classmethod
    def construct_from_string(cls, string):
        if string == cls.name:
            return cls()
        raise TypeError(f"Cannot construct a 'TensorDtype' from '{string}'")

    def __repr__(self):
        return f"TensorDtype(shape={self._shape}, dtype={self._dtype})"

    def __hash__(self):
        return hash((self._shape, self._dtype))

    def __eq__(self, other):
        return isinstance(other, TensorDtype) and other._shape == self._shape and \
            other._dtype == self._dtype

    def __from_arrow__(self, array):
        chunks = array.chunks if isinstance(array, pa.ChunkedArray) else [array]
        return TensorArray(np.concatenate([c.to_numpy() for c in chunks]) if chunks else
                           np.empty((0,) + self._shape, self._dtype))


class TensorArrayElement:
    """One cell of a TensorArray (an ndarray with the column's element shape)."""

    def __init__(self, tensor):
        self._tensor = np.asarray(tensor)

    def to_numpy(self):
        return self._tensor

    def __array__(self, dtype=None, copy=None):
        return self._tensor if dtype is None else self._tensor.astype(dtype)

    def __repr__(self):
        return repr(self._tensor)


class TensorArray(pd.api.extensions.ExtensionArray):
    """A pandas column of equally shaped ndarrays, stored as one (N, *shape) ndarray."""

    def __init__(self, values):
        if isinstance(values, TensorArray):
            values = values._data
        if isinstance(values, (list, tuple)):
            values = np.stack([np.asarray(v.to_numpy() if isinstance(v, TensorArrayElement)
                                          else v) for v in values]) if values else np.empty(0)
        self._data = np.asarray(values)

    @classmethod
    def _from_sequence(cls, scalars, *, dtype=None, copy=False):
        return cls(list(scalars) if not isinstance(scalars, np.ndarray) else scalars)

    @classmethod
    def _from_factorized(cls, values, original):
        return cls(values)

    @classmethod
    def _concat_same_type(cls, to_concat):
        return cls(np.concatenate([t._data for t in to_concat]))

    @property
    def dtype(self):
        return TensorDtype(self._data.shape[1:], self._data.dtype)

    @property
    def nbytes(self):
        return self._data.nbytes

    def __len__(self):
        return self._data.shape[0]

    def __getitem__(self, item):
        if isinstance(item, numbers.Integral):
            return TensorArrayElement(self._data[item])
        return TensorArray(self._data[item])

    def __setitem__(self, key, value):
        self._data[key] = np.asarray(value.to_numpy() if isinstance(value, TensorArrayElement)
                                     else value)

    def isna(self):
        if self._data.dtype.kind == "f":
            return np.isnan(self._data.reshape(len(self), -1)).all(axis=1)
        return np.zeros(len(self), bool)

    def take(self, indices, allow_fill=False, fill_value=None):
        idx = np.asarray(indices)
        if allow_fill:
            out = np.full((len(idx),) + self._data.shape[1:],
                          np.nan if fill_value is None else fill_value,
                          dtype=np.result_type(self._data.dtype, np.float64)
                          if fill_value is None else self._data.dtype)
            ok = idx >= 0
            out[ok] = self._data[idx[ok]]
            return TensorArray(out)
        return TensorArray(self._data.take(idx, axis=0))

    def copy(self):
        return TensorArray(self._data.copy())

    def to_numpy(self, dtype=None, copy=False, na_value=None):
        return self._data if dtype is None else self._data.astype(dtype)

    def __array__(self, dtype=None, copy=None):
        return self.to_numpy(dtype)

    def __arrow_array__(self, type=None):
        return ArrowTensorArray.from_numpy(self._data)

    @property
    def numpy_shape(self):
        return self._data.shape


def column_needs_tensor_extension(s: pd.Series) -> bool:
    """True when a pandas column holds ndarrays (a tensor column)."""
    return s.dtype.type is np.object_ and not s.empty and isinstance(s.iloc[0], np.ndarray)
