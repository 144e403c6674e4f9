"""User API: worker / PS logic contracts, limiters, future-style workers."""
from .futures import BaseMFWorkerLogic, PSClientWithFuture, PullAnswerFuture, WorkerLogicWithFuture
from .limiters import (BlockingPullLimitedWorkerLogic, PullLimitedWorkerLogic, add_blocking_pull_limiter,
                       add_pull_limiter, addBlockingPullLimiter, addPullLimiter)
from .logic import (FunctionWorkerLogic, ParameterServer, ParameterServerClient, ParameterServerLogic,
                    RuntimeContext, WorkerLogic)
