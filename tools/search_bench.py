#!/usr/bin/env python3
"""Search-mode measurements ("Search mode may short-circuit;
report it separately as candidates/sec"), next to bench.py's eval-mode line.

Three numbers, printed as one JSON line:

* ``unsat_candidates_per_s`` -- mg_search (the kernel get_model's GPU
  pre-filter runs, mythril_amd/model.py gpu_search) on a query that no
  candidate satisfies, so every candidate of every chunk is evaluated and
  nothing short-circuits: x*y == 2^255+1 with x, y odd-free (both even);
* ``corpus_batch`` -- mg_batch_search over C2 corpus DAGs (same DAGs as
  bench.py) with 2^20 candidates each: wall time, programs solved, and the
  candidate rate over the candidates actually needed (a solved program stops
  at its first hit, an unsolved one scans all 2^20);
* ``get_model_ms`` -- the drop-in ``get_model`` (reference
  mythril/support/model.py:15-49) on the reference's own satisfiable test
  queries (tests/laser/keccak_tests.py, smt/model_test.py,
  state/calldata_test.py), host flattening + compile + GPU search + witness
  check, median of 5 with the lru cache cleared; and ``batch_is_possible``
  over the same queries as sibling states (one batched search).

* ``shapes`` -- per stand-in query shape C1 / C3 / C4
  (mythril_amd/workloads.py): one batched search over the shape's queries
  (hit rate, candidates/s over the candidates needed, wall time) and the
  drop-in ``get_model`` per query (median latency and the per-phase split:
  flatten, compile, load, search, verify).

Usage:  python tools/search_bench.py [--dags 1024] [--shape-queries 64]
"""

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def reference_sat_queries(engine):
    from mythril_amd.workloads import KeccakFunctionManager as KeccakManager
    from mythril_amd.smt import And, Array, If, symbol_factory
    BVV, BVS = symbol_factory.BitVecVal, symbol_factory.BitVecSym

    def keccak_pair(i1, i2):
        km = KeccakManager(lambda b: engine.keccak256([b])[0])
        o1, c1 = km.create_keccak(i1)
        o2, c2 = km.create_keccak(i2)
        return [And(c1, c2), o1 == o2]
    x = BVS("x", 256)
    cd = Array("1_calldata", 256, 8)
    size = BVS("1_calldatasize", 256)
    return {
        "keccak_same8": keccak_pair(BVV(100, 8), BVV(100, 8)),
        "keccak_sym": keccak_pair(BVS("N1", 256), BVS("N2", 256)),
        "keccak_val_sym": keccak_pair(BVV(100, 256), BVS("N1", 256)),
        "model_x_eq_2": [x == BVV(2, 256)],
        "calldata_byte": [If(BVV(3, 256) < size, cd[BVV(3, 256)], BVV(0, 8)) == BVV(0xA9, 8),
                          size == BVV(4, 256)],
    }


def shape_lines(eng, n_queries, n_sample=48):
    import mythril_amd.model as M
    from mythril_amd import workloads as W
    from mythril_amd.smt.node import topo_order
    out = {}
    M.time_handler.start_execution(3600)
    for name in ("c1", "c3", "c4", "c5"):
        qs = W.queries(name, n_queries)
        M._SEARCH_CACHE = None
        t0 = time.perf_counter()
        progs, qmap = [], []
        for qi, q in enumerate(qs):
            for b in M.dependence_buckets(q):
                progs.append(M._compile_search(b))
                qmap.append(qi)
        t_compile = time.perf_counter() - t0
        loaded = [eng.load(p, M.search_leafgen(p), prog_seed=0) for p in progs]
        n_cand = M.SEARCH_CANDIDATES
        eng.batch_search(loaded[:2], M.SEARCH_SEED, 1 << 16)       # warm-up
        t0 = time.perf_counter()
        hits = eng.batch_search(loaded, M.SEARCH_SEED, n_cand)
        dt = time.perf_counter() - t0
        solved = [True] * len(qs)
        for qi, (i, _) in zip(qmap, hits):
            solved[qi] = solved[qi] and i >= 0
        needed = sum(n_cand if i < 0 else i + 1 for i, _ in hits)
        # recall against the ground-truth labels (tests/golden/recall_labels.json:
        # planted models for SAT, the generator's SafeMath requires for UNSAT)
        recall = None
        lab_path = os.path.join(ROOT, "tests", "golden", "recall_labels.json")
        if os.path.exists(lab_path):
            rows = json.load(open(lab_path))["streams"].get(name, [])
            lab = {r["i"]: r["label"] for r in rows if r["i"] < len(qs)}
            sat = [i for i, l in lab.items() if l == "sat"]
            recall = {"sat_labelled": len(sat), "found": sum(solved[i] for i in sat),
                      "recall": sum(solved[i] for i in sat) / max(1, len(sat)),
                      "missed": [i for i in sat if not solved[i]],
                      "unsat_labelled": sum(l == "unsat" for l in lab.values()),
                      "unsat_found": sum(solved[i] for i, l in lab.items() if l == "unsat"),
                      "unknown_found": sum(solved[i] for i, l in lab.items() if l == "unknown")}
        ins_cand = sum((n_cand if i < 0 else i + 1) * p.n_ins for (i, _), p in zip(hits, progs))
        # the drop-in get_model, one query at a time (no z3 here: a miss
        # raises SolverUnavailable after the GPU search): "cold" compiles
        # every group afresh (16 distinct queries, every memo cleared before
        # each), "stream" keeps the group cache, the group-miss memo and the
        # per-shape statistics across n_sample distinct queries (what
        # successive is_possible calls of one analysis see)
        sample, seen = [], set()
        for q in qs:
            key = tuple(c.id for c in q)
            if key not in seen:
                seen.add(key)
                sample.append(q)
            if len(sample) == n_sample:
                break

        def run(clear_each):
            lat, misses = [], 0
            M.stats.reset_gpu()
            M.clear_search_memos()
            for q in (sample[:16] if clear_each else sample):
                M.get_model.cache_clear()
                if clear_each:
                    M.clear_search_memos()      # compiled groups and group misses
                t1 = time.perf_counter()
                try:
                    M.get_model(tuple(q), enforce_execution_time=False)
                except M.SolverUnavailable:
                    misses += 1
                lat.append((time.perf_counter() - t1) * 1000.0)
            return {"queries": len(lat), "median_ms": statistics.median(lat),
                    "mean_ms": statistics.mean(lat),
                    "max_ms": max(lat), "gpu_misses": misses,
                    "memo_misses": M.stats.memo_misses, "shape_skipped": M.stats.shape_skipped,
                    "gated": M.stats.gated, "kernel_ms_per_query":
                        M.stats.kernel_time * 1000.0 / len(lat),
                    "witness_ms_per_query": M.stats.witness_time * 1000.0 / len(lat),
                    "phase_ms_per_query": {k: v * 1000.0 / len(lat)
                                           for k, v in M.stats.phase.items()}}
        cold = run(True)
        stream = run(False)
        out[name] = {
            "queries": len(qs), "programs": len(progs),
            "source_nodes_mean": statistics.mean(len(topo_order(q)) for q in qs),
            "ir_ins_mean": statistics.mean(p.n_ins for p in progs),
            "compile_ms_per_query": t_compile * 1000.0 / len(qs),
            "batch": {"candidates_per_program": n_cand, "wall_s": dt,
                      "queries_with_witness": sum(solved), "hit_rate": sum(solved) / len(qs),
                      "candidates_needed": needed, "candidates_per_s": needed / dt,
                      "ir_ins_candidates_per_s": ins_cand / dt,
                      # where the witnesses are: how far a search must go
                      "hit_groups": sum(i >= 0 for i, _ in hits),
                      "first_index_max": max([i for i, _ in hits if i >= 0], default=-1),
                      "first_index_over": {str(1 << b): sum(i >= (1 << b) for i, _ in hits)
                                           for b in (8, 12, 16, 18, 20)}},
            "get_model": cold,
            "get_model_stream": stream,
            "recall": recall,
        }
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dags", type=int, default=1024)
    ap.add_argument("--chunks", type=int, default=8, help="2^20-candidate chunks (unsat query)")
    ap.add_argument("--shape-queries", type=int, default=64)
    ap.add_argument("--skip-corpus", action="store_true")
    args = ap.parse_args()

    import bench
    import mythril_amd.model as M
    from mythril_amd.engine import get_engine
    from mythril_amd.ir import compile_constraints
    from mythril_amd.smt import symbol_factory

    corpus = bench.build_corpus(args.dags, min(16, os.cpu_count() or 1))
    eng = get_engine(0)
    out = {"device": eng.device_name}

    # --- unsat query: every candidate evaluated --------------------------
    BVS, BVV = symbol_factory.BitVecSym, symbol_factory.BitVecVal
    x, y = BVS("sx", 256), BVS("sy", 256)
    one = BVV(1, 256)
    cons = [(x & one) == BVV(0, 256), (y & one) == BVV(0, 256), x * y == BVV(2**255 + 1, 256)]
    prog = compile_constraints([c.raw for c in cons],
                               extra_consts=M.harvest_hints([c.raw for c in cons]))
    lp = eng.load(prog, M.search_leafgen(prog), prog_seed=0)
    chunk = 1 << 20
    eng.search(lp, M.SEARCH_SEED, chunk)                      # warm-up
    t0 = time.perf_counter()
    for k in range(args.chunks):
        idx, _ = eng.search(lp, M.SEARCH_SEED, chunk, first_index=k * chunk)
        assert idx < 0, "an even*even product cannot be odd"
    dt = time.perf_counter() - t0
    out["unsat_candidates_per_s"] = args.chunks * chunk / dt
    out["unsat_query"] = {"ir_instructions": int(len(prog.code)), "candidates": args.chunks * chunk,
                          "ms_per_2^20_chunk": dt * 1000.0 / args.chunks}

    out["shapes"] = shape_lines(eng, args.shape_queries)
    print(json.dumps({"shapes": out["shapes"]}), flush=True)
    if args.skip_corpus:
        print(json.dumps(out), flush=True)
        return

    # --- C2 corpus, batched search -----------------------------------------
    loaded = [eng.load(p, M.search_leafgen(p), prog_seed=d) for d, p, _, _ in corpus]
    eng.batch_search(loaded[:8], M.SEARCH_SEED, chunk)         # warm-up
    t0 = time.perf_counter()
    hits = eng.batch_search(loaded, M.SEARCH_SEED, chunk)
    dt = time.perf_counter() - t0
    needed = sum(chunk if i < 0 else i + 1 for i, _ in hits)
    out["corpus_batch"] = {"dags": args.dags, "candidates_per_dag": chunk,
                           "solved": sum(i >= 0 for i, _ in hits), "wall_s": dt,
                           "candidates_needed": needed, "candidates_per_s": needed / dt,
                           "node_candidates_per_s": sum(
                               (chunk if i < 0 else i + 1) * n
                               for (i, _), (_, _, n, _) in zip(hits, corpus)) / dt}

    # --- get_model on the reference's satisfiable test queries --------------
    M.time_handler.start_execution(3600)
    queries = reference_sat_queries(eng)
    lat = {}
    for name, q in queries.items():
        ts = []
        for _ in range(5):
            M.get_model.cache_clear()
            t0 = time.perf_counter()
            M.get_model(tuple(q), enforce_execution_time=False)
            ts.append((time.perf_counter() - t0) * 1000.0)
        lat[name] = statistics.median(ts)
    out["get_model_ms"] = lat
    ts = []
    for _ in range(5):
        M.get_model.cache_clear()
        t0 = time.perf_counter()
        ok = M.batch_is_possible(list(queries.values()), enforce_execution_time=False)
        ts.append((time.perf_counter() - t0) * 1000.0)
        assert ok == [True] * len(queries)
    out["batch_is_possible_ms"] = {"queries": len(queries), "median": statistics.median(ts)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
