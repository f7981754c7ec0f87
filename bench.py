#!/usr/bin/env python3
"""Benchmark: constraint-node evaluations/s on the synthetic corpus (BASELINE
config C2: 4096 random 256-bit DAGs x 2^20 candidate assignments per GPU).

One step = every DAG of the corpus evaluated under 2^20 device-generated
candidates (every node, no short-circuit), root bits written to HBM, the
per-DAG first satisfying candidate reduced with atomicMin and then across
ranks with an RCCL all-reduce(MIN) — the search's one exchange step.
Weak scaling: rank r evaluates candidate indices [r*2^20, (r+1)*2^20) of
every DAG's stream.

``--workload c5`` (config C5) batches every solidity_examples contract's
stand-in query stream (mythril_amd/workloads.py c5_queries: the C1 / C3 / C4
contracts and the other nine) and shards the assignment space like C2, with
the RCCL all-reduce(MIN) of the first witnesses.  ``--shard corpus`` shards
the corpus axis instead: the corpus is ``dags x world`` units, split across
ranks by longest-processing-time first on their DAG sizes
(mythril_amd/shard.py), every rank evaluates its own units' candidates
[s*2^20, (s+1)*2^20) at step s, and nothing is exchanged on the data path
(still weak scaling: per-rank work is one corpus).

Prints ONE JSON line on rank 0 (contract in the task statement).  Extra
fields: roofline (INT32 VALU bound, see mythril_amd/roofline.py) and
cpu_baseline (oracle/evalref.c, the C restatement of z3 model evaluation —
z3 itself is not installed — on host cores, bounded sample).
"""

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SEED = 0x6D797468
# stand-in query streams (mythril_amd/workloads.py): distinct queries per step
STREAM_QUERIES = 256
# LDS spill regions of the batch's context: its register layout's
# (engine.lds_slots_for; MYTHGPU_LDS_SLOTS overrides), set in main() once the
# layout is chosen — the compiled programs are translated for the same
LDS_SLOTS = 6


def explicit_layout():
    """MYTHGPU_NREG, when set: a fixed register layout for every batch of the
    process (A/B runs, the 11-slot parity suite); else None (per-batch rule)."""
    v = os.environ.get("MYTHGPU_NREG")
    return int(v) if v else None


def choose_layout(corpus16, workers, dag_ids, workload, start="fork"):
    """(register slots, corpus compiled for them): the per-batch rule of
    mythril_amd/layout.py over the 16-slot programs (the C2 corpus, whose
    programs barely spill, runs the four-wave layout; the query streams stay
    on 16 slots), recompiled when it picks the four-wave layout."""
    from mythril_amd import layout
    nreg = explicit_layout() or layout.choose([p for _, p, _, _ in corpus16])
    if nreg == 16 and explicit_layout() is None:
        return nreg, corpus16
    return nreg, build_corpus(len(corpus16), workers, dag_ids, workload, start, nreg=nreg)


_STREAM = None


def workload_roots(workload, dag_id):
    """The source DAG (list of root Bools) of unit ``dag_id``: a corpus DAG
    (c2) or the dag_id-th distinct query of a stand-in stream (c3 / c4)."""
    global _STREAM
    if workload == "c2":
        from mythril_amd.corpus import make_dag
        return make_dag(dag_id, SEED)[0]
    if _STREAM is None or _STREAM[0] != workload:
        from mythril_amd import workloads as W
        seen, out = set(), []
        for q in W.queries(workload, 8 * default_units(workload)):
            key = tuple(c.id for c in q)
            if key not in seen:
                seen.add(key)
                out.append(q)
        _STREAM = (workload, out)
    qs = _STREAM[1]
    return qs[dag_id % len(qs)]


def default_units(workload):
    """Units (DAGs / distinct queries) per step: 4096 corpus DAGs (C2), the
    256 distinct queries of a stand-in stream (C3 / C4), 512 distinct queries
    of the all-contracts stream (C5: the thirteen solidity_examples
    contracts, mythril_amd/workloads.py c5_queries)."""
    return {"c2": 4096, "c5": 2 * STREAM_QUERIES}.get(workload, STREAM_QUERIES)


# leaf policy of the eval-mode batch compile: per program ("auto",
# ir.AUTO_SCRATCH_SHARE) unless MYTHRIL_GPU_LEAF_REMAT names one
BENCH_REMAT = os.environ.get("MYTHRIL_GPU_LEAF_REMAT", "auto")


def compile_unit(item):
    """(workload, dag_id[, nreg]) -> (dag_id, Program, node count, int32-op
    weight), compiled for ``nreg`` register slots (default: the process's
    layout, irdefs.NREG)."""
    from mythril_amd import irdefs
    from mythril_amd.ir import compile_constraints
    from mythril_amd.roofline import dag_work
    workload, dag_id = item[:2]
    nreg = item[2] if len(item) > 2 else irdefs.NREG
    roots = workload_roots(workload, dag_id)
    prog = compile_constraints(roots, leaf_remat=BENCH_REMAT, nreg=nreg)
    nodes, weight = dag_work(roots, prog.table_sizes)
    return dag_id, prog, nodes, weight


def build_corpus(n_dags, workers, dag_ids=None, workload="c2", start="fork", nreg=None):
    """Compile the step's DAGs on ``workers`` host processes (fork before
    any GPU initialisation; ``start="spawn"`` from a process that already
    uses the GPU) for ``nreg`` register slots (default: the process's)."""
    from mythril_amd import irdefs
    ids = list(range(n_dags)) if dag_ids is None else list(dag_ids)
    items = [(workload, d, irdefs.NREG if nreg is None else nreg) for d in ids]
    from mythril_amd.procmap import process_map
    return sorted(process_map(compile_unit, items, workers, start, chunksize=16),
                  key=lambda t: t[0])


def programs_digest(corpus) -> str:
    """Digest of the IR programs themselves (instructions and constant
    tables, in DAG order): whichever compiler built them, the same digest
    means the same programs."""
    import hashlib
    h = hashlib.sha1()
    for dag_id, prog, _, _ in sorted(corpus, key=lambda u: u[0]):
        h.update(b"%d:" % dag_id + prog.code.tobytes() + prog.consts.tobytes())
    return h.hexdigest()[:16]


def kernel_key(lib_digest, workload, dags, assign_log2, jit, corpus=None, nreg=None):
    """What a traffic measurement (profiles/traffic.json) is valid for: the
    generated assembly, the allocator's leaf policy, the code path (and for
    compiled programs the digest of the sources that specialise them), the
    workload and the programs evaluated (``programs_digest``).  bench.py
    reports ``traffic`` only when every field matches."""
    from mythril_amd import ir
    key = {"asm_digest": lib_digest, "leaf_remat": BENCH_REMAT, "jit": bool(jit),
           "workload": workload, "dags": dags, "assign_log2": assign_log2}
    if nreg is not None:
        key["nreg"] = nreg
    if corpus is not None:
        key["programs"] = programs_digest(corpus)
    if jit:                           # the compiled programs' own code
        from mythril_amd import jit as J
        key["jit_code"] = J.code_digest()
    return key


def node_image(workload, corpus, workers, world):
    """(compiled-program image of ``corpus``, was it cached).  At world > 1
    the ranks of a node share ONE build (jit.cached_image: the first rank to
    take the file lock assembles with up to 64 host workers, the others wait
    and read it), in ``$MYTHGPU_JIT_CACHE`` or a per-user directory under the
    node's temp dir; at world 1 the image is built in process (timed as
    ``jit_s``) unless ``$MYTHGPU_JIT_CACHE`` is set."""
    import tempfile
    from mythril_amd import jit
    ids = [d for d, _, _, _ in corpus]
    key = "%s_%d_%d_%d_%d_lds%d_r%d" % (workload, len(ids), ids[0], ids[-1], sum(ids), LDS_SLOTS,
                                        corpus[0][1].nreg)
    cache = os.environ.get("MYTHGPU_JIT_CACHE") or (
        os.path.join(tempfile.gettempdir(), "mythgpu_jit_%d" % os.getuid()) if world > 1 else None)
    nw = max(workers, min(os.cpu_count() or 1, 64)) if world > 1 else workers
    return jit.cached_image(key, lambda: jit.compile_batch(
        [(p, None, d) for d, p, _, _ in corpus], workers=nw, lds_slots=LDS_SLOTS), cache)


def same_image(image, world, device=None) -> str:
    """Digest of the image (and of the sources that generate compiled code);
    at world > 1 every rank must hold the same one (assignment axis: all
    ranks run the same programs) — raises otherwise."""
    import hashlib
    from mythril_amd import jit
    dg = hashlib.sha1(image + jit.code_digest().encode()).hexdigest()[:15]
    if world > 1:
        import torch
        import torch.distributed as dist
        v = int(dg, 16)
        t = torch.tensor([v, -v], dtype=torch.int64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if int(t[0]) != v or -int(t[1]) != v:
            raise RuntimeError("ranks hold different compiled-program images (this rank %s)" % dg)
    return dg


def my_dags(mode, n_dags, rank, world, workload="c2"):
    """DAG ids this rank evaluates: every DAG (assignment axis) or its LPT
    share of a ``n_dags x world`` corpus (corpus axis)."""
    if mode == "assign" or world == 1:
        return list(range(n_dags))
    from mythril_amd import shard
    from mythril_amd.corpus import dag_target_nodes
    if workload == "c2":
        costs = [dag_target_nodes(d, SEED) for d in range(n_dags * world)]
    else:                             # stand-in queries: their DAG sizes
        from mythril_amd.smt import node as N
        costs = [len(N.topo_order(workload_roots(workload, d))) for d in range(n_dags * world)]
    return shard.corpus_shard(costs, rank, world)


def step_first(mode, step, rank, world, n_assign):
    """Candidate index of lane 0 at a step: ranks split the candidate space
    (assignment axis) or all scan the same range of disjoint DAGs (corpus)."""
    from mythril_amd import shard
    if mode == "assign":
        return shard.shard_first(step, rank, world, n_assign)
    return shard.shard_first(step, 0, 1, n_assign)


def timed_run(step, sync, steps, warmup, world, device=None):
    """The timed region of the contract: W untimed steps, then K steps
    bracketed by sync + barrier + sync on both sides, elapsed = max over
    ranks.  ``step(i, k)`` runs step i (k = index among the timed steps, or
    None in warmup); ``sync`` waits for this rank's device work."""
    import torch
    import torch.distributed as dist
    for i in range(warmup):
        step(i, None)
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for k in range(steps):
        step(warmup + k, k)
    sync()
    if world > 1:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def all_sum(values, world, device=None):
    """Sum of per-rank numbers (outside the timed region)."""
    if world == 1:
        return list(values)
    import torch
    import torch.distributed as dist
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.tolist()


def sample_indices(corpus):
    """Positions (in the corpus list) of the DAGs the CPU leg times and the
    self-check compares: a stride of 64 over the corpus."""
    return list(range(0, len(corpus), max(1, len(corpus) // 64)))[:64]


def cpu_baseline(corpus, budget_s=20.0, workload="c2", check=None):
    """Time the C restatement oracle on a bounded sample of the same workload
    (same DAGs, same generator) with all host cores.

    ``check`` = (first_index, n_assign, rows, firsts): the GPU's root-bit rows
    (uint64, full width) and per-DAG first satisfying index of the LAST timed
    step for the sampled DAGs.  The oracle then evaluates exactly those
    candidates (indices first_index ...), so the timed CPU work doubles as a
    bit-exact self-check of the timed process's own output: every root bit of
    the sampled prefix, and every first index (consistent with the GPU's full
    row, and checked by the oracle at that lane).  Returns (baseline dict,
    selfcheck dict or None)."""
    from oracle import build as obuild
    from oracle import evalref
    obuild.build()
    # the host-core share (the GPU box exports OMP_NUM_THREADS=16 for one
    # GPU; os.cpu_count() there is the whole machine)
    threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", 0)) or os.cpu_count() or 1, 64))
    first, n_max = (check[0], check[1]) if check is not None else (0, None)
    # calibrate on the first DAG (long enough to amortise thread start-up),
    # then spread the budget over a DAG sample
    sample = [corpus[k] for k in sample_indices(corpus)]
    total_nodes = 0
    t_total = 0.0
    per_dag = None
    outs = []
    for dag_id, prog, nodes, _ in sample:
        roots = workload_roots(workload, dag_id)
        S = evalref.serialize(roots, prog)
        if per_dag is None:
            n_cal = 16384
            t0 = time.perf_counter()
            evalref.run_gen(S, prog, SEED, dag_id, 0, n_cal, threads)
            rate = n_cal * nodes / max(time.perf_counter() - t0, 1e-6)
            per_dag = max(4096, int(rate * budget_s / len(sample) / max(nodes, 1)))
            if n_max is not None:
                per_dag = min(per_dag, n_max)
        t0 = time.perf_counter()
        want = evalref.run_gen(S, prog, SEED, dag_id, first, per_dag, threads)
        t_total += time.perf_counter() - t0
        total_nodes += nodes * per_dag
        outs.append((dag_id, prog, S, want))
    base = {"value": total_nodes / t_total, "unit": "node-evals/s", "cores": threads,
            "kind": "port",
            "sample": "%d %s DAGs x %d generated assignments (%.3g node-evals, %.1f s); "
                      "oracle/evalref.c restates z3 model evaluation (z3 not installed)"
                      % (len(sample), workload, per_dag, total_nodes, t_total)}
    if check is None:
        return base, None
    from mythril_amd.engine import unpack_bits
    _, n_assign, rows, firsts = check
    bad_bits = bad_first = 0
    for (dag_id, prog, S, want), row, f in zip(outs, rows, firsts):
        got = unpack_bits(row, n_assign)
        bad_bits += int(np.count_nonzero(got[:per_dag] != want))
        hit = np.flatnonzero(got)
        gpu_first = first + int(hit[0]) if hit.size else -1
        if int(f) != gpu_first:                   # d_first disagrees with the bits
            bad_first += 1
        elif hit.size and int(hit[0]) >= per_dag:  # beyond the compared prefix:
            if not evalref.run_gen(S, prog, SEED, dag_id, gpu_first, 1, threads)[0]:
                bad_first += 1                    # the oracle must agree at that lane
    sc = {"dags": len(outs), "lanes": per_dag, "first_index": first,
          "mismatches": bad_bits, "first_sat_mismatches": bad_first,
          "what": "last timed step: root bits of %d sampled units x %d candidates and their "
                  "first satisfying index vs oracle/evalref.c" % (len(outs), per_dag)}
    return base, sc


def waves_per_simd(nreg: int) -> int:
    """Waves per SIMD the layout's VGPR budget allows (512 per lane)."""
    from mythril_amd import asmgen
    with asmgen.layout(nreg):
        return 512 // asmgen.NVGPR_KERNEL


def engine_lib_path() -> str:
    from mythril_amd import engine
    return engine._LIB_PATH


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=("c2", "c3", "c4", "c5"), default="c2",
                    help="c2: synthetic corpus (default, BASELINE configs[1]); c3 / c4: the "
                         "BECToken / token+WalletLibrary stand-in query streams; c5: every "
                         "solidity_examples contract's stream, batched (configs[4])")
    ap.add_argument("--dags", type=int, default=None,
                    help="DAGs per step (default 4096 for c2, %d distinct queries for c3/c4, "
                         "%d for c5)" % (STREAM_QUERIES, 2 * STREAM_QUERIES))
    ap.add_argument("--assign-log2", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--shard", choices=("assign", "corpus"), default="assign",
                    help="assignment axis (default, C2) or corpus axis (C5)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"))
    ap.add_argument("--interp", action="store_true",
                    help="record dispatch through the assembly interpreter instead of the "
                         "compiled programs (mythril_amd/jit.py, the default)")
    ap.add_argument("--jit", action="store_true", help=argparse.SUPPRESS)  # the default
    ap.add_argument("--jit-build-only", action="store_true",
                    help="compile the corpus and its code object into $MYTHGPU_JIT_CACHE and "
                         "exit (no GPU): profiling runs then load it")
    args = ap.parse_args()
    args.jit = not args.interp
    if args.dags is None:
        args.dags = default_units(args.workload)

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    # host-side corpus compile (before any GPU initialisation, so fork is safe)
    ncpu = os.cpu_count() or 1
    # (MYTHGPU_BENCH_WORKERS: profiled runs, where every forked worker also
    # carries the profiler's GPU context, keep the process count low)
    workers = int(os.environ.get("MYTHGPU_BENCH_WORKERS", "0")) or \
        max(1, min(16, ncpu // max(1, world)))
    t0 = time.time()
    mine = my_dags(args.shard, args.dags, rank, world, args.workload)
    corpus16 = build_corpus(args.dags, workers, mine, args.workload, nreg=16)
    # the batch's register layout (mythril_amd/layout.py): chosen from the
    # 16-slot programs, recompiled for it when it is the four-wave one
    nreg, corpus = choose_layout(corpus16, workers, mine, args.workload)
    from mythril_amd import layout as LAY
    progs16 = [p for _, p, _, _ in corpus16]
    layout_rule = {"nreg": nreg, "rule": "four waves when the 16-slot programs average >= %.2f "
                   "heavy records and <= %.1f scratch spill slots (mythril_amd/layout.py)"
                   % (LAY.W4_MIN_HEAVY_SHARE, LAY.W4_MAX_SCRATCH_SLOTS),
                   "mean_scratch_slots_16": round(LAY.mean_scratch_slots(progs16), 3),
                   "mean_heavy_share_16": round(LAY.mean_heavy_share(progs16), 4),
                   "explicit": explicit_layout() is not None}
    del corpus16, progs16
    global LDS_SLOTS
    from mythril_amd.engine import lds_slots_for
    LDS_SLOTS = lds_slots_for(nreg)
    t_compile = time.time() - t0
    image, t_jit, jit_cached = None, 0.0, False
    if args.jit:                      # code generation + assembly, still before the GPU
        t0 = time.time()
        image, jit_cached = node_image(args.workload, corpus, workers, world)
        t_jit = time.time() - t0
    if args.jit_build_only:
        print("jit image %.1f MB in %.1f s (cached: %s)" % (len(image or b"") / 1e6, t_jit,
                                                          jit_cached), flush=True)
        return

    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", local))

    from mythril_amd import shard
    from mythril_amd.engine import Engine, default_leafgen
    image_digest = None
    if image is not None:                     # assignment axis: every rank runs the same code
        image_digest = same_image(image, world if args.shard == "assign" else 1, "cuda")
    eng = Engine(local, nreg=nreg)
    loaded = [eng.load(p, default_leafgen(p), prog_seed=d) for d, p, _, _ in corpus]
    if image is not None:
        jit_handle = eng.jit_attach(loaded, image)     # noqa: F841 (kept attached)
    batch = eng.batch_create(loaded)
    n_assign = 1 << args.assign_log2
    words = (n_assign + 63) // 64
    n_mine = len(corpus)
    d_bits = torch.empty((n_mine, words), dtype=torch.int64, device="cuda")
    d_first = torch.empty(n_mine, dtype=torch.int64, device="cuda")
    # a dedicated (non-default) stream: the library launches on exactly this
    # stream, so the HIP events below bracket the kernel itself (a null
    # handle would make the library fall back to its own internal stream)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    nodes_per_lane = sum(n for _, _, n, _ in corpus)
    weight_per_lane = sum(w for _, _, _, w in corpus)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]

    def step(i, k):
        d_first.fill_(shard.NONE)
        first = step_first(args.shard, i, rank, world, n_assign)
        if k is not None:
            evs[k][0].record(stream)
        eng.batch_eval_gen(batch, SEED, first, n_assign, d_bits.data_ptr(), d_first.data_ptr(),
                           stream.cuda_stream)
        if k is not None:
            evs[k][1].record(stream)
        if args.shard == "assign":
            shard.reduce_first_sat(d_first)  # the one exchange step (RCCL MIN)

    elapsed = timed_run(step, torch.cuda.synchronize, args.steps, args.warmup, world, "cuda")
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / args.steps
    sat_local = int((d_first != shard.NONE).sum().item())
    nodes_all, weight_all, sat_all = all_sum([nodes_per_lane, weight_per_lane, sat_local],
                                             world, "cuda")
    if args.shard == "assign":
        nodes_all, sat_all = nodes_per_lane * world, sat_local     # every rank: every DAG
    sat_dags = int(sat_all)

    if rank == 0:
        from mythril_amd.roofline import VALU_PEAK_OPS
        ms_step = elapsed * 1000.0 / args.steps
        evals = nodes_all * n_assign * args.steps
        ops_launch = weight_per_lane * n_assign
        achieved = ops_launch / (kern_ms / 1000.0)
        key = kernel_key(eng.lib.mg_asm_digest_layout(nreg).decode(), args.workload, args.dags,
                         args.assign_log2, args.jit, corpus, nreg)
        traffic, traffic_note, sq = None, "no profiles/traffic.json", None
        if os.path.exists(args.traffic_json):
            try:
                with open(args.traffic_json) as fh:
                    tj = json.load(fh)
                entries = tj.get("entries", [tj] if "kernel_key" in tj else [])
                hit = next((e for e in entries if e.get("kernel_key") == key), None)
                if hit is not None:
                    traffic = hit.get("hbm_bytes_per_launch")
                    sq = hit.get("sq")
                    traffic_note = ("rocprofv3 FETCH_SIZE x2 + WRITE_SIZE per launch of this "
                                    "kernel (profiles/traffic.json entry with the same "
                                    "kernel_key, %s)" % hit.get("evidence", "profiles/"))
                else:
                    same = [e["kernel_key"] for e in entries
                            if e.get("kernel_key", {}).get("workload") == args.workload]
                    diff = sorted(k for k in key if (same[0] if same else {}).get(k) != key[k])
                    traffic_note = "profiles/traffic.json has no entry for this kernel (%s " \
                        "differ)" % ", ".join(diff)
            except (OSError, ValueError) as e:
                traffic_note = "profiles/traffic.json unreadable: %s" % e
        workload_txt = {
            "c2": "C2 synthetic corpus: %d random 256-bit DAGs (64-512 nodes)" % args.dags,
            "c3": "C3 stand-in stream: %d distinct BECToken-shaped integer-overflow queries "
                  "(mythril_amd/workloads.py)" % args.dags,
            "c4": "C4 stand-in stream: %d distinct token + WalletLibrary keccak/mapping queries "
                  "(mythril_amd/workloads.py)" % args.dags,
            "c5": "C5 all-contracts stream: %d distinct queries of the 13 solidity_examples "
                  "contracts' stand-in streams, batched (mythril_amd/workloads.py c5_queries)"
                  % args.dags}[args.workload]
        out = {
            "metric": "constraint-node evals/sec",
            "value": evals / elapsed,
            "unit": "node-evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32x8 (256-bit bit-vectors)",
            "data": "synthetic (corpus seed 0x6d797468, device-generated candidates)",
            "config": {"workload": ("%s x 2^%d assignments per GPU" % (workload_txt, args.assign_log2))
                       if args.shard == "assign" else
                       ("corpus axis: %s per GPU, LPT-sharded by DAG size, x 2^%d assignments "
                        "each" % (workload_txt, args.assign_log2)),
                       "dags": args.dags * (world if args.shard == "corpus" else 1),
                       "assignments_per_gpu": n_assign, "nodes_total": int(nodes_all),
                       "shard": args.shard, "parallelism": "dp%d" % world,
                       "register_layout": "%d slots, %d waves/SIMD, %d LDS regions"
                                          % (nreg, waves_per_simd(nreg), LDS_SLOTS),
                       "layout_rule": layout_rule},
            "roofline": {"bound": "valu", "achieved": achieved / 1e12, "peak": VALU_PEAK_OPS / 1e12,
                         "unit": "Tops/s (int32 VALU)", "frac": achieved / VALU_PEAK_OPS,
                         "traffic": traffic, "traffic_note": traffic_note, "kernel_ms": kern_ms,
                         "int32_ops_per_launch": ops_launch,
                         # the executed-instruction view (SQ pass of this same
                         # kernel_key, profiles/traffic.json "sq"): VALU lane-
                         # instructions issued per second against the same
                         # peak, and the share of SIMD cycles issuing VALU
                         "valu_issue": (sq["valu_insts"] * 64 / (kern_ms / 1000.0) / VALU_PEAK_OPS
                                        if sq and sq.get("valu_insts") else None),
                         "valu_active": sq.get("valu_active") if sq else None,
                         "valu_insts_per_node_eval": (sq["valu_insts"] * 64 /
                                                      (nodes_per_lane * n_assign)
                                                      if sq and sq.get("valu_insts") else None)},
            "kernel_key": key,
            "runtime": dict(eng.runtime_info(), library=os.path.basename(engine_lib_path()),
                            torch_hip=getattr(torch.version, "hip", None),
                            note="the library's NEEDED libamdhip64.so.7 binds to the runtime "
                                 "torch loaded first (tests/test_gpu_torch_runtime.py checks "
                                 "parity in that configuration)"),
            "sat_dags": sat_dags,
            "compile_s": round(t_compile, 2),
            "path": "compiled programs (mythril_amd/jit.py)" if args.jit else "interpreter",
            "jit_s": round(t_jit, 2) if args.jit else None,
            "jit_cached": jit_cached if args.jit else None,
            "jit_image_digest": image_digest,
        }
        if world == 1 and not args.no_cpu_baseline:
            last = step_first(args.shard, args.warmup + args.steps - 1, rank, world, n_assign)
            pos = sample_indices(corpus)
            idx = torch.tensor(pos, dtype=torch.long, device="cuda")
            rows = d_bits.index_select(0, idx).cpu().numpy().view(np.uint64)
            firsts = d_first.index_select(0, idx).cpu().numpy()
            firsts = np.where(firsts == shard.NONE, -1, firsts)
            out["cpu_baseline"], out["selfcheck"] = cpu_baseline(
                corpus, workload=args.workload, check=(last, n_assign, rows, firsts))
            out["vs_cpu"] = out["value"] / out["cpu_baseline"]["value"]
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
