"""Multi-GPU sharding of the witness search.

The units — (DAG, candidate index) pairs — are independent, so both axes
shard with no data-path collective:

* **assignment axis** (one process per GPU; ``bench.py`` default): at step
  ``s`` rank ``r`` of ``world`` evaluates the candidate indices
  ``[(s*world + r) * n, (s*world + r + 1) * n)`` of every DAG's counter-based
  stream (the device generator regenerates any candidate from its index, so
  witnesses are never gathered).  The single exchange step is the per-DAG
  first satisfying index, reduced with MIN across ranks
  (``torch.distributed`` all-reduce: RCCL over xGMI on GPUs, gloo on CPU).
  ``NONE`` (INT64_MAX) means "no witness".
* **corpus axis** (config C5; ``bench.py --shard corpus``, and
  ``model.batch_is_possible`` over several devices of one process): whole
  DAGs are assigned to ranks / devices by longest-processing-time first on
  an estimated cost (:func:`lpt_assign`), each evaluates its DAGs' full
  candidate range, and nothing is exchanged at all (a DAG's first witness
  is found on the one device that owns it).

The reference has no distributed code at all (Mythril is
single-process); this axis is the one the engine creates.
"""

from __future__ import annotations

from typing import List, Tuple

NONE = 0x7FFFFFFFFFFFFFFF


def shard_first(step: int, rank: int, world: int, n_assign: int) -> int:
    """First candidate index rank ``rank`` evaluates at ``step``."""
    if not (0 <= rank < world) or n_assign <= 0 or step < 0:
        raise ValueError("bad shard (step=%d rank=%d world=%d n=%d)" % (step, rank, world, n_assign))
    return (step * world + rank) * n_assign


def shard_ranges(step: int, world: int, n_assign: int) -> List[Tuple[int, int]]:
    """[first, last) of every rank at ``step`` (disjoint, contiguous)."""
    return [(shard_first(step, r, world, n_assign), shard_first(step, r, world, n_assign) + n_assign)
            for r in range(world)]


def reduce_first_sat(first_sat, group=None) -> None:
    """In-place MIN all-reduce of a per-DAG int64 first-satisfying-index
    tensor across the ranks of ``group`` (no-op for a single process)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(first_sat, op=dist.ReduceOp.MIN, group=group)


def lpt_assign(costs: List[float], world: int) -> List[List[int]]:
    """Corpus axis (config C5): longest-processing-time-first assignment of
    DAGs (estimated cost = weight x candidates) to ``world`` ranks; each
    rank's list is sorted, the lists partition ``range(len(costs))``, and the
    heaviest rank carries at most the lightest rank's load plus one DAG."""
    import heapq
    if world <= 0:
        raise ValueError("world must be positive")
    heap = [(0.0, r) for r in range(world)]
    out: List[List[int]] = [[] for _ in range(world)]
    for i in sorted(range(len(costs)), key=lambda k: (-costs[k], k)):
        load, r = heapq.heappop(heap)
        out[r].append(i)
        heapq.heappush(heap, (load + costs[i], r))
    for lst in out:
        lst.sort()
    return out


def corpus_shard(costs: List[float], rank: int, world: int) -> List[int]:
    """The DAG indices rank ``rank`` owns on the corpus axis."""
    if not (0 <= rank < world):
        raise ValueError("bad rank %d of %d" % (rank, world))
    return lpt_assign(costs, world)[rank]
