"""``ray.data.preprocessor`` (reference: python/ray/data/preprocessor.py): the
``Preprocessor`` base class (implementations in data/preprocessors.py)."""

from ray_amd.data.preprocessors import (Preprocessor,  # noqa: F401
                                        PreprocessorNotFittedException)

__all__ = ["Preprocessor", "PreprocessorNotFittedException"]
