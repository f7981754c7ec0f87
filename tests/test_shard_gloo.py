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
