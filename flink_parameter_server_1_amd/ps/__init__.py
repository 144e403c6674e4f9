"""PS-side logic library (per-record) and HBM-resident device tables."""
from .logics import (IllegalStateException, LockPSLogicA, LockPSLogicB, RangePSLogicWithClose, SimplePSLogic,
                     SimplePSLogicWithClose, range_shard_bounds)
