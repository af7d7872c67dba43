"""``ray.rllib.utils.typing`` (reference path): the type aliases RLlib signatures use."""

from typing import Any, Callable, Dict, List, Tuple, Union

import numpy as np

TensorType = Any
TensorStructType = Union[TensorType, dict, tuple, list]
TensorShape = Union[Tuple[int, ...], List[int]]
AgentID = Any
PolicyID = str
ModuleID = str
EnvID = Any
EpisodeID = Union[int, str]
EnvType = Any
EnvConfigDict = dict
EnvCreator = Callable[[dict], Any]
AlgorithmConfigDict = dict
PartialAlgorithmConfigDict = dict
ModelConfigDict = dict
ResultDict = dict
LearningRateOrSchedule = Union[float, List[List[Union[int, float]]]]
MultiAgentDict = Dict[AgentID, Any]
MultiEnvDict = Dict[EnvID, MultiAgentDict]
SampleBatchType = Any
StateDict = Dict[str, Any]
ModelWeights = dict
ModelGradients = Union[List[TensorType], List[tuple]]
TensorStructType = TensorStructType
FileType = Any
SpaceStruct = Any
ViewRequirementsDict = dict
LocalOptimizer = Any
Optimizer = Any
ParamDict = dict
NetworkType = Any
DeviceType = Any
NDArray = np.ndarray
