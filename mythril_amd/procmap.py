"""Order-preserving process map that fails fast when a worker dies.

``multiprocessing.Pool.map`` never returns when a worker process is killed
(an abort in native code — the round-4 ``stack smashing detected`` in the
oracle workers of tests/test_gpu_bench_parity.py — leaves the pool waiting
for a result that will not come, until pytest's timeout kills the whole GPU
run).  ``concurrent.futures.ProcessPoolExecutor`` notices the dead process
and raises ``BrokenProcessPool`` for every pending item at once, so the
caller fails within seconds with the cause in the log."""

from concurrent.futures import ProcessPoolExecutor
from concurrent.futures.process import BrokenProcessPool  # noqa: F401 - re-exported
from typing import Callable, Iterable, List


def process_map(fn: Callable, items: Iterable, workers: int, start: str = "fork",
                chunksize: int = 1) -> List:
    """``[fn(x) for x in items]`` on ``workers`` processes of the ``start``
    method (``fork`` before any GPU initialisation, ``spawn`` from a process
    that already holds the GPU).  Raises ``BrokenProcessPool`` as soon as a
    worker dies; any exception a worker raises is re-raised here."""
    import multiprocessing as mp
    items = list(items)
    if workers <= 1 or len(items) <= 1:
        return [fn(x) for x in items]
    with ProcessPoolExecutor(max_workers=min(workers, len(items)),
                             mp_context=mp.get_context(start)) as ex:
        return list(ex.map(fn, items, chunksize=max(1, chunksize)))
