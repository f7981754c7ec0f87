"""Lists the C2 corpus DAGs with satisfying lanes in candidates [2^20, 2^20 + 2^16)
(the slice tests/test_gpu_parity.py::test_bench_entry_point_bit_exact_against_c_oracle
checks); run on a GPU box."""
import sys, os
sys.path.insert(0, os.getcwd())
import bench, torch
from mythril_amd.engine import Engine, default_leafgen
from mythril_amd import shard
corpus = bench.build_corpus(4096, 16)
torch.cuda.set_device(0)
eng = Engine(0)
loaded = [eng.load(p, default_leafgen(p), prog_seed=d) for d, p, _, _ in corpus]
b = eng.batch_create(loaded)
n, first = 1 << 16, 1 << 20
d_bits = torch.zeros((4096, n // 64), dtype=torch.int64, device="cuda")
d_first = torch.full((4096,), shard.NONE, dtype=torch.int64, device="cuda")
eng.batch_eval_gen(b, bench.SEED, first, n, d_bits.data_ptr(), d_first.data_ptr())
torch.cuda.synchronize()
f = d_first.cpu().tolist()
print("SAT", [(d, f[d] - first) for d in range(4096) if f[d] != shard.NONE])
