"""Tensor extension types (reference: python/ray/data/extensions/__init__.py)."""

from ray_amd.data.extensions.tensor_extension import (  # noqa: F401
    ArrowTensorArray, ArrowTensorType, ArrowVariableShapedTensorArray,
    ArrowVariableShapedTensorType, TensorArray, TensorArrayElement, TensorDtype,
    column_needs_tensor_extension)

__all__ = ["TensorDtype", "TensorArray", "TensorArrayElement", "ArrowTensorType",
           "ArrowTensorArray", "ArrowVariableShapedTensorType",
           "ArrowVariableShapedTensorArray", "column_needs_tensor_extension"]
