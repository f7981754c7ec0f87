"""SMT-LIB 2 capture / replay: dump -> parse gives the
same hash-consed constraints, z3-style text (let, #x, _i divisions, as const,
UF) parses, and the recorder logs get_model calls for the replay census."""

import json

import pytest

import dag_cases
import mythril_amd.model as M
from mythril_amd import capture, smtlib
from mythril_amd.corpus import make_dag
from mythril_amd.smt import ULT, node as N, symbol_factory


@pytest.mark.parametrize("name", sorted(dag_cases.named_cases()))
def test_dump_parse_round_trip_cases(name):
    constraints, probes, _, _ = dag_cases.named_cases()[name]
    cs = list(constraints) + [p for p in probes if p.is_bool()]
    back = smtlib.parse_query(smtlib.dump_query(cs))
    assert len(back) == len(cs) and all(a is b for a, b in zip(cs, back))


def test_dump_parse_round_trip_corpus():
    for d in (0, 3, 17, 99):
        roots, _ = make_dag(d, 0x6D797468)
        text = smtlib.dump_query(roots)
        assert "define-fun" in text                 # shared sub-terms named once
        back = smtlib.parse_query(text)
        # corpus DAGs live in their own hash-consing scope (corpus.make_dag),
        # so the parsed nodes are equal in structure, not the same objects
        assert len(back) == len(roots)
        assert smtlib.dump_query(back) == text


def test_parse_z3_style_text():
    text = """; produced by Solver.sexpr()
(declare-fun x () (_ BitVec 256))
(declare-fun |1_calldata| () (Array (_ BitVec 256) (_ BitVec 8)))
(declare-fun keccak256_256 ((_ BitVec 256)) (_ BitVec 256))
(assert (let ((a!1 (bvudiv_i x #x0000000000000000000000000000000000000000000000000000000000000002)))
  (and (= (select |1_calldata| (_ bv3 256)) #xa9) (bvule a!1 (keccak256_256 x))
       (= ((_ extract 7 0) a!1) #b00000001))))
(assert (= (select ((as const (Array (_ BitVec 256) (_ BitVec 256))) #x0000000000000000000000000000000000000000000000000000000000000000) x) x))
(check-sat)
"""
    got = smtlib.parse_query(text)
    x = N.bv_var("x", 256)
    cd = N.array_var("1_calldata", 256, 8)
    q = N.bv_op("bvudiv", x, N.bv_num(2, 256))
    want0 = N.bool_op("and", N.eq(N.select(cd, N.bv_num(3, 256)), N.bv_num(0xA9, 8)),
                      N.bv_cmp("bvule", q, N.apply_uf("keccak256_256", 256, 256, x)),
                      N.eq(N.extract(7, 0, q), N.bv_num(1, 8)))
    want1 = N.eq(N.select(N.const_array(256, N.bv_num(0, 256)), x), x)
    assert got == [want0, want1]


def test_parse_errors_are_reported():
    with pytest.raises(smtlib.ParseError):
        smtlib.parse_query("(assert (bvadd y y))")
    with pytest.raises(smtlib.ParseError):
        smtlib.parse_query("(assert (= x")


def test_recorder_logs_outcomes_and_census(tmp_path, monkeypatch):
    M.get_model.cache_clear()
    monkeypatch.setattr(M.z3bridge, "available", lambda: False)

    def fake_search(nodes, budget_ms):
        return None if any(n.op == "false" for n in nodes) else (M.Assignment(vars={"x": 1}), None)
    monkeypatch.setattr(M, "gpu_search", fake_search)

    def fake_z3(constraints, minimize, maximize, timeout):
        raise M.UnsatError
    monkeypatch.setattr(M, "_z3_check", fake_z3)
    M.args.solver_timeout = 10000
    M.time_handler.start_execution(3600)
    path = str(tmp_path / "q.jsonl")
    rec = capture.Recorder(path, M.get_model)
    x = symbol_factory.BitVecSym("x", 256)
    sat = (ULT(x, symbol_factory.BitVecVal(5, 256)),)
    unsat = (symbol_factory.Bool(False).__class__(symbol_factory.Bool(False).raw),)
    rec(sat)
    with pytest.raises(M.UnsatError):
        rec(unsat)
    with pytest.raises(M.UnsatError):
        rec(sat + (False,))
    rows = capture.read(path)
    assert [r["result"] for r in rows] == ["sat", "unsat", "unsat"]
    assert rows[2]["python_bools"] == [False]
    assert smtlib.parse_query(rows[0]["smt2"])[0] is sat[0].raw
    c = capture.census(rows)
    assert c["queries"] == 3 and c["compiled"] == 3 and c["ops"]["bvult"] == 2
    M.get_model.cache_clear()


def test_cli_replay_census(tmp_path, capsys):
    path = tmp_path / "q.jsonl"
    roots, _ = make_dag(4, 0x6D797468)
    path.write_text(json.dumps({"id": 0, "minimize": 0, "maximize": 0, "python_bools": [],
                                "smt2": smtlib.dump_query(roots), "result": "sat"}) + "\n")
    assert capture.main(["replay", str(path)]) == 0
    out = json.loads(capsys.readouterr().out)
    assert out["census"]["compiled"] == 1 and out["census"]["nodes"] > 60
