"""Multi-process (world_size 2, gloo on CPU) coverage of the N>1 witness-search
path bench.py runs over RCCL: candidate-space sharding + the MIN all-reduce
of per-DAG first satisfying indices (mythril_amd/shard.py).

Each rank evaluates its shard with the C oracle (tests only) standing in for
the GPU launch; the reduced result must equal a single-process sweep of the
whole range."""

import os
import socket

import numpy as np
import pytest

from mythril_amd import shard
from mythril_amd.ir import compile_constraints
from mythril_amd.smt import node as N

SEED = 0x6D797468
N_ASSIGN = 96


def _dags():
    x, y = N.bv_var("x", 256), N.bv_var("y", 256)
    lo = N.extract(3, 0, x)
    return [
        [N.bv_cmp("bvult", x, y)],                                        # ~1/2
        [N.eq(lo, N.bv_num(5, 4)), N.bv_cmp("bvult", y, x)],              # ~1/32
        [N.eq(N.extract(11, 0, N.bv_op("bvxor", x, y)), N.bv_num(0xABC, 12))],  # ~0 in range
        [N.bv_cmp("bvule", N.bv_op("bvmul", x, y), x)],
    ]


def _local_first(dag_id, roots, first, n):
    from oracle import evalref
    prog = compile_constraints(roots)
    S = evalref.serialize(roots, prog)
    sat = evalref.run_gen(S, prog, SEED, dag_id, first, n, threads=1)
    idx = np.flatnonzero(sat)
    return first + int(idx[0]) if idx.size else shard.NONE


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dags = _dags()
        res = []
        for step in range(2):
            first = shard.shard_first(step, rank, world, N_ASSIGN)
            local = torch.tensor([_local_first(d, r, first, N_ASSIGN) for d, r in enumerate(dags)],
                                 dtype=torch.int64)
            shard.reduce_first_sat(local)
            res.append(local.tolist())
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_ranges_partition():
    for world in (1, 2, 3, 8):
        for step in range(3):
            rs = shard.shard_ranges(step, world, 1 << 10)
            assert rs[0][0] == step * world * (1 << 10)
            for (a0, a1), (b0, _) in zip(rs, rs[1:]):
                assert a1 == b0
            assert rs[-1][1] - rs[0][0] == world * (1 << 10)
    with pytest.raises(ValueError):
        shard.shard_first(0, 2, 2, 8)


def test_lpt_assign_balances():
    costs = [9, 7, 6, 5, 4, 3, 2, 2, 1]
    parts = shard.lpt_assign(costs, 3)
    assert sorted(i for p in parts for i in p) == list(range(len(costs)))
    loads = [sum(costs[i] for i in p) for p in parts]
    assert max(loads) - min(loads) <= max(costs)


def test_gloo_world2_first_sat_matches_single_process():
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[0] == out[1]                      # every rank holds the reduced result
    dags = _dags()
    for step in range(2):
        lo = step * world * N_ASSIGN
        want = [_local_first(d, r, lo, world * N_ASSIGN) for d, r in enumerate(dags)]
        assert out[0][step] == want
    assert out[0][0][0] != shard.NONE            # the easy DAG is found in every step


# ---- corpus axis (C5) and bench.py's world > 1 timed loop -----------------

def test_corpus_shard_partitions_and_balances():
    from mythril_amd.corpus import dag_target_nodes, make_dag
    import bench
    for world in (2, 3, 8):
        parts = [bench.my_dags("corpus", 64, r, world) for r in range(world)]
        assert sorted(i for p in parts for i in p) == list(range(64 * world))
        costs = [dag_target_nodes(d) for d in range(64 * world)]
        loads = [sum(costs[i] for i in p) for p in parts]
        assert max(loads) - min(loads) <= max(costs)
    assert bench.my_dags("assign", 16, 1, 4) == list(range(16))
    for d in (0, 5, 77):                               # the estimate is the DAG's own draw
        roots, n = make_dag(d)
        assert n >= dag_target_nodes(d) and n <= dag_target_nodes(d) + 8
    # corpus axis: every rank scans the same candidate range of its own DAGs
    assert bench.step_first("corpus", 3, 1, 4, 1 << 20) == 3 << 20
    assert bench.step_first("assign", 3, 1, 4, 1 << 20) == (3 * 4 + 1) << 20


def _bench_worker(rank, world, port, q):
    """bench.py's own timed loop and reductions at world 2 over gloo, with the
    engine launch replaced by the C oracle on this rank's shard (CPU)."""
    import time
    import torch
    import torch.distributed as dist
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dags = _dags()
        firsts = {}
        first_sat = torch.full((len(dags),), shard.NONE, dtype=torch.int64)

        def step(i, k):
            first_sat.fill_(shard.NONE)
            first = bench.step_first("assign", i, rank, world, N_ASSIGN)
            first_sat.copy_(torch.tensor([_local_first(d, r, first, N_ASSIGN)
                                          for d, r in enumerate(dags)], dtype=torch.int64))
            if rank == 1:
                time.sleep(0.2)                       # the slow rank sets the clock
            shard.reduce_first_sat(first_sat)
            firsts[i] = first_sat.tolist()

        elapsed = bench.timed_run(step, lambda: None, steps=2, warmup=1, world=world)
        nodes, sat = bench.all_sum([10.0 + rank, float(rank)], world)
        q.put((rank, elapsed, firsts, nodes, sat))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_bench_timed_loop_world2_gloo(world):
    """(world 4: the N > 2 reductions the driver's scaling runs take, on CPU)"""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {r: (e, f, n, s) for r, e, f, n, s in (q.get(timeout=240) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # elapsed is the max over ranks (the slow rank's two timed steps), on all
    assert len({out[r][0] for r in range(world)}) == 1 and out[0][0] >= 0.4
    # warmup step 0 and timed steps 1, 2: reduced first witnesses equal a
    # single-process sweep over every rank's range
    dags = _dags()
    for i in range(3):
        lo = i * world * N_ASSIGN
        want = [_local_first(d, r, lo, world * N_ASSIGN) for d, r in enumerate(dags)]
        assert all(out[r][1][i] == want for r in range(world))
    nodes, sat = sum(10.0 + r for r in range(world)), float(sum(range(world)))
    assert all(out[r][2] == nodes and out[r][3] == sat for r in range(world))


def _image_worker(rank, world, port, q, cache_dir):
    """bench.py's node-shared compiled-program image at world 2: both ranks
    ask for the same corpus's image; one builds it under the file lock, the
    other reads it, and the digest check across ranks passes — and fails on
    both ranks when one holds a different image."""
    import torch.distributed as dist
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["MYTHGPU_JIT_CACHE"] = cache_dir
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        corpus = bench.build_corpus(3, 1)
        image, cached = bench.node_image("c2", corpus, 1, world)
        dg = bench.same_image(image, world)
        refused = False
        try:
            bench.same_image(image + (b"x" if rank == 1 else b""), world)
        except RuntimeError:
            refused = True
        q.put((rank, cached, dg, refused))
    finally:
        dist.destroy_process_group()


def test_bench_shares_one_image_per_node_world2_gloo(tmp_path):
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_image_worker, args=(r, world, port, q, str(tmp_path)))
             for r in range(world)]
    for p in procs:
        p.start()
    out = {r: (c, d, f) for r, c, d, f in (q.get(timeout=300) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert sorted(out[r][0] for r in out) == [False, True]      # built once, read once
    assert out[0][1] == out[1][1]
    assert out[0][2] and out[1][2]                              # a differing rank is refused
    assert len([f for f in os.listdir(tmp_path) if f.endswith(".hsaco")]) == 1
