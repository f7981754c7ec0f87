"""mythril_amd.procmap: the process map used for the bench / JIT builds and
the GPU tests' oracle workers fails fast when a worker dies (VERDICT r4 item
6: an aborting oracle worker hung ``multiprocessing.Pool.map`` until
pytest-timeout killed a metered GPU run)."""

import os
import time

import pytest

from mythril_amd.procmap import BrokenProcessPool, process_map


def _square(x):
    return x * x


def _abort_on_3(x):
    if x == 3:
        os.abort()                       # what a native crash looks like to the pool
    return x


def _raise_on_2(x):
    if x == 2:
        raise ValueError("bad item %d" % x)
    return x


@pytest.mark.parametrize("start", ["fork", "spawn"])
def test_order_and_values(start):
    assert process_map(_square, range(37), 4, start, chunksize=3) == [x * x for x in range(37)]


def test_a_dying_worker_fails_within_seconds():
    t0 = time.monotonic()
    with pytest.raises(BrokenProcessPool):
        process_map(_abort_on_3, range(64), 4, "spawn", chunksize=2)
    assert time.monotonic() - t0 < 30


def test_a_worker_exception_is_reraised():
    with pytest.raises(ValueError, match="bad item 2"):
        process_map(_raise_on_2, range(8), 3, "fork")


def test_serial_below_two_workers():
    assert process_map(_square, [1, 2, 3], 1) == [1, 4, 9]
