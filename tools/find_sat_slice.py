"""Lists the C2 corpus DAGs with satisfying lanes in candidates
[2^20, 2^20 + 2^16) (the slice tests/test_gpu_parity.py::
test_bench_entry_point_bit_exact_against_c_oracle checks), with the C oracle
on host cores (no GPU).  Rerun whenever the candidate generator changes."""
import os
import sys

sys.path.insert(0, os.getcwd())
import bench  # noqa: E402
from oracle import evalref  # noqa: E402

THREADS = int(os.environ.get("OMP_NUM_THREADS", "0")) or os.cpu_count() or 1
corpus = bench.build_corpus(4096, min(16, os.cpu_count() or 1))
n, first = 1 << 16, 1 << 20
sat = []
for d, p, _, _ in corpus:
    roots = bench.workload_roots("c2", d)
    bits = evalref.run_gen(evalref.serialize(roots, p), p, bench.SEED, d, first, n, THREADS)
    if bits.any():
        sat.append((d, int(bits.argmax())))
print("SAT", sat)
