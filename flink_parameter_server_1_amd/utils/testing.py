"""Success-exception test harness (C50, ``T/test/utils/FlinkTestUtils.scala:8-29``).

A Flink job has no return value, so the reference's tests end a job from a
sink: the sink's ``close()`` throws ``SuccessException(result)``; the harness
runs ``env.execute()``, digs the ``SuccessException`` out of the
``JobExecutionException`` cause chain and runs a checker on the result.

Here a job is any callable (usually a ``transform`` call with
``runtime=LocalRuntime(output_sink=sink)``); ``LocalRuntime.close`` calls the
sink's ``close()``, so the same pattern works unchanged.
"""
from __future__ import annotations

from typing import Any, Callable, List, Optional


class SuccessException(Exception):
    def __init__(self, result: Any = None):
        super().__init__("job finished successfully")
        self.result = result


def _find_success(exc: Optional[BaseException]) -> Optional[SuccessException]:
    seen = set()
    while exc is not None and id(exc) not in seen:
        if isinstance(exc, SuccessException):
            return exc
        seen.add(id(exc))
        exc = exc.__cause__ or exc.__context__
    return None


def execute_with_success_check(job: Callable[[], Any], check: Optional[Callable[[Any], None]] = None) -> Any:
    """Run ``job``; it must end by raising ``SuccessException`` (possibly wrapped).
    Runs ``check(result)`` and returns the result.  Any other failure propagates;
    a job that ends normally is a failed test, as in the reference."""
    try:
        job()
    except BaseException as e:  # noqa: BLE001 - unwrap like the reference harness
        ok = _find_success(e)
        if ok is None:
            raise
        if check is not None:
            check(ok.result)
        return ok.result
    raise AssertionError("job finished without SuccessException")


class CollectingSuccessSink:
    """Sink collecting every output; ``close()`` ends the job with the collected list
    (optionally transformed by ``finish``)."""

    def __init__(self, finish: Optional[Callable[[List[Any]], Any]] = None):
        self.items: List[Any] = []
        self.finish = finish

    def __call__(self, e):
        self.items.append(e)

    def close(self):
        raise SuccessException(self.finish(self.items) if self.finish else list(self.items))
