"""bench.py's self-check (CPU): the CPU-baseline leg evaluates the sampled
units on exactly the candidates of the last timed step and compares the
GPU's root-bit rows and first indices with them.  Here the "GPU" rows are
made by the oracle itself, then corrupted, to show every kind of mismatch is
counted."""

import numpy as np

import bench
from mythril_amd import shard
from oracle import evalref


def _rows(corpus, first, n):
    rows, firsts = [], []
    for k in bench.sample_indices(corpus):
        d, p, _, _ = corpus[k]
        want = evalref.run_gen(evalref.serialize(bench.workload_roots("c2", d), p), p, bench.SEED,
                               d, first, n, 2)
        rows.append(np.packbits(want, bitorder="little").view(np.uint64))
        hit = np.flatnonzero(want)
        firsts.append(first + int(hit[0]) if hit.size else -1)
    return np.array(rows), np.array(firsts, dtype=np.int64)


def test_selfcheck_counts_bit_and_first_index_mismatches():
    corpus = bench.build_corpus(6, 1)
    n, first = 1 << 13, 3 << 20
    rows, firsts = _rows(corpus, first, n)
    base, sc = bench.cpu_baseline(corpus, budget_s=5.0, check=(first, n, rows, firsts))
    assert base["kind"] == "port" and base["value"] > 0
    assert sc["dags"] == 6 and sc["lanes"] == n and sc["first_index"] == first
    assert sc["mismatches"] == 0 and sc["first_sat_mismatches"] == 0
    bad = rows.copy()
    bad[2, 5] ^= np.uint64(1 << 7)                # one root bit
    bad_f = firsts.copy()
    bad_f[4] = first + 5 if firsts[4] < 0 else firsts[4] + 1      # one first index
    _, sc = bench.cpu_baseline(corpus, budget_s=5.0, check=(first, n, bad, bad_f))
    assert sc["mismatches"] == 1
    assert sc["first_sat_mismatches"] >= 1


def test_selfcheck_verifies_a_first_index_beyond_the_compared_prefix(monkeypatch):
    """When the budget covers fewer lanes than the step, a first index past
    the prefix is checked by the oracle at that one lane."""
    corpus = bench.build_corpus(3, 1)
    n, first = 1 << 13, 7 << 20
    rows, firsts = _rows(corpus, first, n)
    real = evalref.run_gen
    calls = []

    def spy(S, prog, seed, ps, f, m, threads=0, pct=(50, 70, 85)):
        calls.append((f, m))
        return real(S, prog, seed, ps, f, m, threads, pct)
    monkeypatch.setattr(evalref, "run_gen", spy)
    # a first set bit at lane 5000, past the 4096-lane minimum prefix
    rows[0, 5000 // 64] |= np.uint64(1 << (5000 % 64))
    firsts[0] = first + 5000 if firsts[0] < 0 else firsts[0]
    _, sc = bench.cpu_baseline(corpus, budget_s=0.0, check=(first, n, rows, firsts))
    assert sc["lanes"] == 4096
    if firsts[0] == first + 5000:
        assert (first + 5000, 1) in calls            # the one-lane oracle check ran
        d, p, _, _ = corpus[0]
        sat = real(evalref.serialize(bench.workload_roots("c2", d), p), p, bench.SEED, d,
                   first + 5000, 1, 1)[0]
        assert sc["first_sat_mismatches"] == (0 if sat else 1)
    assert shard.NONE > 0
