"""hyperspace_amd — an MI355X-native covering-index query engine with the capabilities of
Microsoft Hyperspace (reference: pirz/hyperspace-1).

Host side: Python metadata/optimizer layers + a C++ runtime (``csrc/runtime``); device side:
hand-written HIP/CDNA4 kernels (``csrc/kernels``) for bucketing, radix partition/sort, predicate
scans, bucket-local joins and aggregation; multi-GPU via torch.distributed (RCCL over xGMI).
"""
from .exceptions import HyperspaceException, NoChangesException
from .hyperspace import Hyperspace, get_context
from .index.config import IndexConfig
from .session import Session
from .plan.column import col, lit, sum_, count, min_, max_, avg

__all__ = ["Hyperspace", "IndexConfig", "Session", "HyperspaceException", "NoChangesException",
           "col", "lit", "sum_", "count", "min_", "max_", "avg", "get_context"]

__version__ = "0.1.0"
