"""z3-free mirror of ``mythril.laser.smt`` — the expression vocabulary of the
``get_model`` hot path.

Every class and helper here builds the same DAG shape the reference builds
with z3 (operator → SMT-LIB op mapping cited per function), so the IR
compiler sees exactly the node kinds LASER hands to ``get_model``:

* ``BitVec`` operators: ``mythril/laser/smt/bitvec.py:63-253``
  (``/`` is **bvsdiv**, ``<``/``>``/``<=``/``>=`` are **signed**, ``>>`` is
  **bvashr**, ``==``/``!=`` zero-pad the narrower side, ``bitvec.py:16-22``).
* helpers ``If/UGT/ULT/UGE/ULE/Concat/Extract/URem/SRem/UDiv/Sum/LShR`` and the
  ``BV*NoOverflow`` predicates: ``mythril/laser/smt/bitvec_helper.py:21-214``
  (``UGE = Or(UGT, ==)`` and ``ULE = Or(ULT, ==)``, ``:53-80``).
* ``Bool``/``And``/``Or``/``Xor``/``Not``: ``mythril/laser/smt/bool.py:14-141``.
* ``Array``/``K``: ``mythril/laser/smt/array.py:16-63``;
  ``Function``: ``mythril/laser/smt/function.py:7-25``.
* ``symbol_factory``: ``mythril/laser/smt/__init__.py:83-154``.

``simplify`` is structural only (it returns the expression unchanged):
evaluation never happens on the host — DAGs are evaluated by the HIP engine.
"""

from __future__ import annotations

from typing import Any, Iterable, List, Optional, Set, Union

from . import node as N
from .node import Node

Annotations = Set[Any]


class Expression:
    """Base of BitVec/Bool (reference ``expression.py:10-55``)."""

    def __init__(self, raw: Node, annotations: Optional[Annotations] = None):
        if not isinstance(raw, Node):
            raise TypeError("raw must be a DAG node")
        self.raw = raw
        if annotations:
            assert isinstance(annotations, set)
        self._annotations = annotations or set()

    @property
    def annotations(self) -> Annotations:
        return self._annotations

    def annotate(self, annotation: Any) -> None:
        self._annotations.add(annotation)

    def simplify(self) -> None:
        """Structural no-op (z3's rewriter is not reproduced on the host)."""

    def size(self) -> int:
        return self.raw.width

    def get_annotations(self, annotation: Any):
        return [a for a in self.annotations if isinstance(a, annotation)]

    def __repr__(self) -> str:
        return repr(self.raw)

    def __hash__(self) -> int:
        return hash(self.raw)


def simplify(expression):
    expression.simplify()
    return expression


def _num(value: int, width: int) -> Node:
    return N.bv_num(value, width)


def _padded(a: Node, b: Node):
    """``_padded_operation`` (``bitvec.py:16-22``): zero-extend the narrower
    operand by concatenating a zero numeral on the left."""
    if a.width == b.width:
        return a, b
    swapped = a.width < b.width
    big, small = (b, a) if swapped else (a, b)
    small = N.concat(_num(0, big.width - small.width), small)
    return (small, big) if swapped else (big, small)


class Bool(Expression):
    """Boolean expression (``bool.py:14-92``)."""

    @property
    def is_false(self) -> bool:
        return self.raw.op == "false"

    @property
    def is_true(self) -> bool:
        return self.raw.op == "true"

    @property
    def value(self) -> Optional[bool]:
        if self.is_true:
            return True
        if self.is_false:
            return False
        return None

    def __eq__(self, other) -> "Bool":  # type: ignore[override]
        if isinstance(other, Expression):
            return Bool(N.eq(self.raw, other.raw), self.annotations.union(other.annotations))
        return Bool(N.eq(self.raw, N.bool_val(bool(other))), self.annotations)

    def __ne__(self, other) -> "Bool":  # type: ignore[override]
        if isinstance(other, Expression):
            return Bool(N.distinct(self.raw, other.raw), self.annotations.union(other.annotations))
        return Bool(N.distinct(self.raw, N.bool_val(bool(other))), self.annotations)

    def __bool__(self) -> bool:
        v = self.value
        return v if v is not None else False

    def __hash__(self) -> int:
        return hash(self.raw)


def _as_bool(a: Union[Bool, bool]) -> Bool:
    return a if isinstance(a, Bool) else Bool(N.bool_val(bool(a)))


def And(*args: Union[Bool, bool]) -> Bool:
    items = [_as_bool(a) for a in args]
    ann: Set = set()
    for a in items:
        ann = ann.union(a.annotations)
    return Bool(N.bool_op("and", *[a.raw for a in items]), ann)


def Or(*args: Union[Bool, bool]) -> Bool:
    items = [_as_bool(a) for a in args]
    ann: Set = set()
    for a in items:
        ann = ann.union(a.annotations)
    return Bool(N.bool_op("or", *[a.raw for a in items]), ann)


def Xor(a: Bool, b: Bool) -> Bool:
    return Bool(N.bool_op("xor", a.raw, b.raw), a.annotations.union(b.annotations))


def Not(a: Bool) -> Bool:
    return Bool(N.bool_op("not", a.raw), a.annotations)


def is_true(a: Bool) -> bool:
    return a.raw.op == "true"


def is_false(a: Bool) -> bool:
    return a.raw.op == "false"


class BitVec(Expression):
    """Bit-vector expression (``bitvec.py:25-253``)."""

    def size(self) -> int:
        return self.raw.width

    @property
    def symbolic(self) -> bool:
        return self.raw.op != "bvnum"

    @property
    def value(self) -> Optional[int]:
        return self.raw.params[0] if self.raw.op == "bvnum" else None

    def _other(self, other) -> "BitVec":
        return other if isinstance(other, BitVec) else BitVec(_num(other, self.size()))

    def _arith(self, op: str, other) -> "BitVec":
        o = self._other(other)
        return BitVec(N.bv_op(op, self.raw, o.raw), self.annotations.union(o.annotations))

    def __add__(self, other):
        return self._arith("bvadd", other)

    def __sub__(self, other):
        return self._arith("bvsub", other)

    def __mul__(self, other):
        return self._arith("bvmul", other)

    def __truediv__(self, other):
        return self._arith("bvsdiv", other)   # bitvec.py:96-103: signed division

    def __and__(self, other):
        return self._arith("bvand", other)

    def __or__(self, other):
        return self._arith("bvor", other)

    def __xor__(self, other):
        return self._arith("bvxor", other)

    def _cmp(self, op: str, other) -> Bool:
        o = self._other(other)
        return Bool(N.bv_cmp(op, self.raw, o.raw), self.annotations.union(o.annotations))

    def __lt__(self, other):
        return self._cmp("bvslt", other)      # bitvec.py:138-148: signed

    def __gt__(self, other):
        return self._cmp("bvsgt", other)

    def __le__(self, other):
        return self._cmp("bvsle", other)

    def __ge__(self, other):
        return self._cmp("bvsge", other)

    def __eq__(self, other) -> Bool:  # type: ignore[override]
        if not isinstance(other, BitVec):
            return Bool(N.eq(self.raw, _num(other, self.size())), self.annotations)
        a, b = _padded(self.raw, other.raw)
        return Bool(N.eq(a, b), self.annotations.union(other.annotations))

    def __ne__(self, other) -> Bool:  # type: ignore[override]
        if not isinstance(other, BitVec):
            return Bool(N.distinct(self.raw, _num(other, self.size())), self.annotations)
        a, b = _padded(self.raw, other.raw)
        return Bool(N.distinct(a, b), self.annotations.union(other.annotations))

    def _shift(self, op: str, other) -> "BitVec":
        o = self._other(other)
        return BitVec(N.bv_op(op, self.raw, o.raw), self.annotations.union(o.annotations))

    def __lshift__(self, other):
        return self._shift("bvshl", other)

    def __rshift__(self, other):
        return self._shift("bvashr", other)   # z3 '>>' on BitVecRef is arithmetic

    def __hash__(self) -> int:
        return hash(self.raw)


def _ann(*xs) -> Set:
    out: Set = set()
    for x in xs:
        out = out.union(x.annotations)
    return out


def LShR(a: BitVec, b: BitVec) -> BitVec:
    return BitVec(N.bv_op("bvlshr", a.raw, b.raw), _ann(a, b))


def If(a: Union[Bool, bool], b: Union[BitVec, int], c: Union[BitVec, int]) -> BitVec:
    a = _as_bool(a)
    if not isinstance(b, BitVec):
        b = BitVec(_num(b, 256))
    if not isinstance(c, BitVec):
        c = BitVec(_num(c, 256))
    return BitVec(N.ite(a.raw, b.raw, c.raw), _ann(a, b, c))


def UGT(a: BitVec, b: BitVec) -> Bool:
    return Bool(N.bv_cmp("bvugt", a.raw, b.raw), _ann(a, b))


def ULT(a: BitVec, b: BitVec) -> Bool:
    return Bool(N.bv_cmp("bvult", a.raw, b.raw), _ann(a, b))


def UGE(a: BitVec, b: BitVec) -> Bool:
    return Or(UGT(a, b), a == b)      # bitvec_helper.py:53-62


def ULE(a: BitVec, b: BitVec) -> Bool:
    return Or(ULT(a, b), a == b)      # bitvec_helper.py:73-80


def Concat(*args) -> BitVec:
    bvs: List[BitVec] = list(args[0]) if len(args) == 1 and isinstance(args[0], list) else list(args)
    return BitVec(N.concat(*[a.raw for a in bvs]), _ann(*bvs))


def Extract(high: int, low: int, bv: BitVec) -> BitVec:
    return BitVec(N.extract(high, low, bv.raw), bv.annotations)


def URem(a: BitVec, b: BitVec) -> BitVec:
    return BitVec(N.bv_op("bvurem", a.raw, b.raw), _ann(a, b))


def SRem(a: BitVec, b: BitVec) -> BitVec:
    return BitVec(N.bv_op("bvsrem", a.raw, b.raw), _ann(a, b))


def UDiv(a: BitVec, b: BitVec) -> BitVec:
    return BitVec(N.bv_op("bvudiv", a.raw, b.raw), _ann(a, b))


def Sum(*args: BitVec) -> BitVec:
    acc = args[0].raw
    for a in args[1:]:
        acc = N.bv_op("bvadd", acc, a.raw)
    return BitVec(acc, _ann(*args))


def _bv256(x) -> BitVec:
    return x if isinstance(x, BitVec) else BitVec(_num(x, 256))


def BVAddNoOverflow(a, b, signed: bool) -> Bool:
    """z3's unsigned add-no-overflow: the carry bit of the (w+1)-bit sum is 0."""
    a, b = _bv256(a), _bv256(b)
    if signed:
        raise NotImplementedError("signed BVAddNoOverflow is not used by Mythril")
    w = a.size()
    s = N.bv_op("bvadd", N.zero_extend(1, a.raw), N.zero_extend(1, b.raw))
    return Bool(N.eq(N.extract(w, w, s), _num(0, 1)))


def BVMulNoOverflow(a, b, signed: bool) -> Bool:
    a, b = _bv256(a), _bv256(b)
    if signed:
        raise NotImplementedError("signed BVMulNoOverflow is not used by Mythril")
    return Bool(N.bv_cmp("bvumul_noovfl", a.raw, b.raw))


def BVSubNoUnderflow(a, b, signed: bool) -> Bool:
    """z3's unsigned sub-no-underflow is ``bvule(b, a)``."""
    a, b = _bv256(a), _bv256(b)
    if signed:
        raise NotImplementedError("signed BVSubNoUnderflow is not used by Mythril")
    return Bool(N.bv_cmp("bvule", b.raw, a.raw))


class BaseArray:
    """``array.py:16-37``: Select/Store; a Bool stored becomes If(v, 1, 0)."""

    raw: Node

    def __getitem__(self, item: BitVec) -> BitVec:
        if isinstance(item, slice):
            raise ValueError("Instance of BaseArray, does not support getitem with slices")
        return BitVec(N.select(self.raw, item.raw))

    def __setitem__(self, key: BitVec, value) -> None:
        if isinstance(value, Bool):
            value = If(value, 1, 0)
        self.raw = N.store(self.raw, key.raw, value.raw)


class Array(BaseArray):
    def __init__(self, name: str, domain: int, value_range: int):
        self.domain = domain
        self.range = value_range
        self.raw = N.array_var(name, domain, value_range)


class K(BaseArray):
    def __init__(self, domain: int, value_range: int, value: int):
        self.domain = domain
        self.range = value_range
        self.value = _num(value, value_range)
        self.raw = N.const_array(domain, self.value)


class Function:
    """Uninterpreted function of one bit-vector argument (``function.py``)."""

    def __init__(self, name: str, domain: int, value_range: int):
        self.name = name
        self.domain = domain
        self.range = value_range

    def __call__(self, item: BitVec) -> BitVec:
        return BitVec(N.apply_uf(self.name, self.domain, self.range, item.raw),
                      annotations=item.annotations)


class _SymbolFactory:
    """``symbol_factory`` (reference ``laser/smt/__init__.py:83-154``)."""

    @staticmethod
    def Bool(value: bool, annotations: Optional[Annotations] = None) -> Bool:
        return Bool(N.bool_val(value), annotations)

    @staticmethod
    def BoolSym(name: str, annotations: Optional[Annotations] = None) -> Bool:
        return Bool(N.bool_var(name), annotations)

    @staticmethod
    def BitVecVal(value: int, size: int, annotations: Optional[Annotations] = None) -> BitVec:
        return BitVec(_num(value, size), annotations)

    @staticmethod
    def BitVecSym(name: str, size: int, annotations: Optional[Annotations] = None) -> BitVec:
        return BitVec(N.bv_var(name, size), annotations)


symbol_factory = _SymbolFactory()

__all__ = [
    "Expression", "BitVec", "Bool", "And", "Or", "Xor", "Not", "is_true", "is_false",
    "If", "UGT", "ULT", "UGE", "ULE", "Concat", "Extract", "URem", "SRem", "UDiv", "Sum",
    "LShR", "BVAddNoOverflow", "BVMulNoOverflow", "BVSubNoUnderflow", "BaseArray", "Array",
    "K", "Function", "symbol_factory", "simplify", "Node",
]


def raws(exprs: Iterable[Expression]) -> List[Node]:
    return [e.raw for e in exprs]
