"""Pin the C restatement (oracle/evalref.c, used for big CPU sweeps and the
cpu_baseline leg) to the Python oracle on every test case."""

import random

import pytest

import dag_cases
from mythril_amd.assign import Assignment as PAssignment, leaf_values, unpack
from mythril_amd.corpus import make_dag
from mythril_amd.ir import compile_constraints
from oracle import evalref, gen_ref
from oracle import smtlib_ref as R

CASES = dag_cases.named_cases()


@pytest.mark.parametrize("name", sorted(CASES))
def test_c_oracle_matches_python_oracle(name):
    constraints, probes, gen, tables = CASES[name]
    prog = compile_constraints(constraints, probes, table_sizes=tables)
    S = evalref.serialize(constraints, prog, probes)
    rng = random.Random(77)
    asgs = [gen(rng) for _ in range(80)]
    lvs = [leaf_values(prog, PAssignment(a.vars, a.arrays, a.funcs)) for a in asgs]
    roots, vals = evalref.run_leaves(S, prog, lvs, want_nodes=True)
    for a, asg in enumerate(asgs):
        want = R.evaluate(list(probes), asg)
        got = [evalref.node_value(vals, a, S.node_index[p.id]) for p in probes]
        assert got == want, (name, a)
        assert bool(roots[a]) == bool(R.eval_constraints(constraints, asg))


@pytest.mark.parametrize("dag_id", [0, 3, 17, 256])
def test_c_oracle_generator_matches(dag_id):
    roots, _ = make_dag(dag_id)
    prog = compile_constraints(roots)
    S = evalref.serialize(roots, prog)
    bits = evalref.run_gen(S, prog, 0xC0FFEE, dag_id, 1000, 40, threads=2)
    for a in range(40):
        lv = [gen_ref.gen_leaf(0xC0FFEE, dag_id, li, 1000 + a, l.width, prog.const_values)
              for li, l in enumerate(prog.leaves)]
        import numpy as np
        arr = np.zeros((len(lv), 8), dtype=np.uint32)
        for i, v in enumerate(lv):
            for j in range(8):
                arr[i, j] = (v >> (32 * j)) & 0xFFFFFFFF
        asg = unpack(prog, arr)
        assert bool(bits[a]) == bool(R.eval_constraints(roots, R.Assignment(asg.vars, asg.arrays, asg.funcs)))
