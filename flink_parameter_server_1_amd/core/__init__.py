"""Messages, partitioners, wire adapters and the per-record engines."""
from .adapters import *  # noqa: F401,F403
from .engine import (FlinkParameterServer, LocalRuntime, LogicFactory, PartitionedInput, transform,
                     transform_with_double_model_load, transform_with_model_load)
from .messages import Either, Left, Pull, PullAnswer, Push, PSToWorker, Right, WorkerToPS, left_values, right_values
from .partitioners import (HashPartitioner, Partitioner, RangePartitioner, hash_partition, range_partition,
                           range_partitioner_ps)
