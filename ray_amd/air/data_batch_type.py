"""The batch types Predictors and map_batches accept (reference: air/data_batch_type.py)."""
from typing import Dict, Union

import numpy as np

try:
    import pandas as _pd

    DataBatchType = Union[np.ndarray, _pd.DataFrame, Dict[str, np.ndarray]]
except ImportError:  # pragma: no cover
    DataBatchType = Union[np.ndarray, Dict[str, np.ndarray]]
