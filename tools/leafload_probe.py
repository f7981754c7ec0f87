#!/usr/bin/env python3
"""Diagnostic (round 6): what the leaf generator's memory classes cost a
stand-in workload.  The default class mix (engine.default_leafgen: 50 %
uniform, 20 % small, 15 % boundary-table loads, 15 % pool loads) against mixes
without the loads, same programs, compiled code, one kernel per variant
(alternated twice).  Not a bench line: the candidate distribution IS part of
the workload; this only prices the loads' latency.
usage: tools/leafload_probe.py [workload] [units]"""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    w = sys.argv[1] if len(sys.argv) > 1 else "c3"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else bench.default_units(w)
    from mythril_amd import jit
    from mythril_amd.engine import default_leafgen, get_engine, lds_slots_for
    nreg, corpus = bench.choose_layout(bench.build_corpus(n, 16, workload=w, nreg=16), 16, None, w)
    print("layout %d slots" % nreg, flush=True)
    variants = {"base": (50, 70, 85), "noload": (50, 100, 100), "bnd_only": (50, 70, 100),
                "pool_only": (50, 85, 85)}
    images = {}
    for k, pct in variants.items():
        t0 = time.time()
        images[k] = jit.compile_batch([(p, default_leafgen(p, pct), d) for d, p, _, _ in corpus],
                                      workers=16, lds_slots=lds_slots_for(nreg))
        print("image %s %.1f s" % (k, time.time() - t0), flush=True)
    import torch
    eng = get_engine(0, nreg=nreg)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    n_assign = 1 << 20
    d_bits = torch.empty((len(corpus), n_assign // 64), dtype=torch.int64, device="cuda")
    d_first = torch.empty(len(corpus), dtype=torch.int64, device="cuda")
    res = {k: [] for k in variants}
    for rnd in range(2):
        for k, pct in variants.items():
            loaded = [eng.load(p, default_leafgen(p, pct), prog_seed=d) for d, p, _, _ in corpus]
            h = eng.jit_attach(loaded, images[k])
            batch = eng.batch_create(loaded)
            for rep in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                d_first.fill_(-1)
                e0.record(stream)
                eng.batch_eval_gen(batch, bench.SEED, (rep + 1) << 20, n_assign, d_bits.data_ptr(),
                                   d_first.data_ptr(), stream.cuda_stream)
                e1.record(stream)
                torch.cuda.synchronize()
                if rep:
                    res[k].append(e0.elapsed_time(e1))
            eng.batch_free(batch)
            eng.jit_detach(h)
            del loaded
            print("round %d %-10s %s ms %s" % (rnd, k, ["%.2f" % x for x in res[k][-2:]], pct),
                  flush=True)
    base = min(res["base"])
    for k in variants:
        print("%-10s best %.2f ms  (%.1f %% of base)" % (k, min(res[k]), 100.0 * min(res[k]) / base))


if __name__ == "__main__":
    main()
