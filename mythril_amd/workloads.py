"""Shape-faithful stand-ins for the captured-query configs of BASELINE.json
(C1 ``suicide.sol -t 2``, C3 ``BECToken.sol -t 3`` integer-overflow checks,
C4 ``WalletLibrary.sol`` + ``token.sol`` mapping/storage constraints).

These are NOT captured queries: capturing needs z3 and solc, which exist on
neither this container nor the GPU box.  Each query is built
with the z3-free ``laser.smt`` mirror (:mod:`mythril_amd.smt`) by replaying,
opcode handler by opcode handler, the lowering LASER applies on the path a
function call takes through the contract's compiled dispatcher:

* transaction setup — ``sender_{N}`` constrained to the three actors
  (``transaction/symbolic.py:165-167``), ``UGE(balance[sender], call_value{N})``
  and the balance transfer store chain (``transaction_models.py:121-133``);
* calldata — ``{N}_calldata`` (256 -> 8) and ``{N}_calldatasize``; a word is
  ``Concat`` of 32 ``If(off + i < size, calldata[off + i], 0)`` with the
  SIGNED ``<`` of ``BitVec.__lt__`` (``calldata.py:47-54,219-232``);
* dispatcher — ``Not(ULT(calldatasize, 4))``, the selector
  ``0xffffffff & UDiv(word(0), 2**224)`` compared with each function id
  (``instructions.py:480-490,330-352,716-740``), a JUMPI appending ``condi`` or
  ``Not(condi)`` (``instructions.py:1543-1619``), ISZERO as ``If(.., 1, 0)``
  (``:743-760``) so a BitVec JUMPI condition becomes ``x != 0``;
* mappings — ``sha3`` of ``Concat(key, slot)`` as the keccak UF pair with the
  interval / mod-64 / known-hash condition (``keccak_function_manager.py:
  83-149``, ``instructions.py:1010-1048``; concrete data hashed on the host),
  read and written through the ``Storage{addr}`` store chain
  (``state/account.py:18-82``; ``K(256, 256, 0)`` after a creation
  transaction);
* overflow checks — ``Not(BVAddNoOverflow)``, ``Not(BVMulNoOverflow)``,
  ``Not(BVSubNoUnderflow)`` on the operands of ADD / MUL / SUB, appended to
  the path constraints at the transaction end exactly as the integer module
  poses them (``analysis/module/modules/integer.py:143-157,268-280``).

z3's ``simplify`` is not reproduced (``smt.simplify`` is structural), so the
DAGs carry LASER's pre-simplification shapes.  Every query is a list of Bool
DAG nodes, the argument ``get_model`` receives.
"""

from __future__ import annotations

import random
from typing import Dict, List, Optional, Sequence, Tuple

from . import smt as S
from .smt import node as N

# ---------------------------------------------------------------------------
# host Keccak-256 for concrete hash data (keccak_function_manager.py:43-57
# hashes concrete inputs on the host with ethereum.utils.sha3)
# ---------------------------------------------------------------------------

_RC = [0x0000000000000001, 0x0000000000008082, 0x800000000000808A, 0x8000000080008000,
       0x000000000000808B, 0x0000000080000001, 0x8000000080008081, 0x8000000000008009,
       0x000000000000008A, 0x0000000000000088, 0x0000000080008009, 0x000000008000000A,
       0x000000008000808B, 0x800000000000008B, 0x8000000000008089, 0x8000000000008003,
       0x8000000000008002, 0x8000000000000080, 0x000000000000800A, 0x800000008000000A,
       0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008]
_ROT = [[0, 36, 3, 41, 18], [1, 44, 10, 45, 2], [62, 6, 43, 15, 61], [28, 55, 25, 21, 56],
        [27, 20, 39, 8, 14]]
_M = (1 << 64) - 1


def _rol(x: int, n: int) -> int:
    return ((x << n) | (x >> (64 - n))) & _M if n else x


def keccak256(data: bytes) -> bytes:
    """Keccak-256 (original 0x01 padding, as Ethereum uses)."""
    rate = 136
    msg = bytearray(data) + b"\x01" + b"\x00" * ((-len(data) - 1) % rate)
    msg[-1] |= 0x80
    st = [[0] * 5 for _ in range(5)]
    for off in range(0, len(msg), rate):
        for i in range(rate // 8):
            st[i % 5][i // 5] ^= int.from_bytes(msg[off + 8 * i: off + 8 * i + 8], "little")
        for rc in _RC:
            c = [st[x][0] ^ st[x][1] ^ st[x][2] ^ st[x][3] ^ st[x][4] for x in range(5)]
            d = [c[(x - 1) % 5] ^ _rol(c[(x + 1) % 5], 1) for x in range(5)]
            st = [[st[x][y] ^ d[x] for y in range(5)] for x in range(5)]
            b = [[0] * 5 for _ in range(5)]
            for x in range(5):
                for y in range(5):
                    b[y][(2 * x + 3 * y) % 5] = _rol(st[x][y], _ROT[x][y])
            st = [[b[x][y] ^ (~b[(x + 1) % 5][y] & b[(x + 2) % 5][y]) for y in range(5)]
                  for x in range(5)]
            st[0][0] ^= rc
    return b"".join(st[i % 5][i // 5].to_bytes(8, "little") for i in range(4))


def selector(signature: str) -> int:
    return int.from_bytes(keccak256(signature.encode())[:4], "big")


# ---------------------------------------------------------------------------
# keccak UF pairs (keccak_function_manager.py:24-149)
# ---------------------------------------------------------------------------

TOTAL_PARTS = 10 ** 40
PART = (2 ** 256 - 1) // TOTAL_PARTS
INTERVAL_DIFFERENCE = 10 ** 30


class KeccakFunctionManager:
    """``KeccakFunctionManager``: ``keccak256_N`` / ``keccak256_N-1`` UF pairs,
    one interval ``[idx*PART, idx*PART + PART)`` per input width, outputs
    ``= 0 mod 64``, and an ``Or`` over every concrete hash seen so far."""

    def __init__(self, hasher=keccak256):
        self.hasher = hasher
        self.store_function: Dict[int, Tuple[S.Function, S.Function]] = {}
        self.interval_hook_for_size: Dict[int, int] = {}
        self._index_counter = TOTAL_PARTS - 34534
        self.concrete_hashes: Dict[S.BitVec, S.BitVec] = {}
        self.hash_result_store: Dict[int, List[S.BitVec]] = {}

    def get_function(self, length: int):
        if length not in self.store_function:
            self.store_function[length] = (S.Function("keccak256_{}".format(length), length, 256),
                                           S.Function("keccak256_{}-1".format(length), 256, length))
            self.hash_result_store[length] = []
        return self.store_function[length]

    def get_concrete_hash_data(self, model) -> Dict[int, List[int]]:
        """``keccak_function_manager.py:103-119``: the model's values of every
        symbolic hash created so far, per input size."""
        out: Dict[int, List[int]] = {}
        for size, vals in self.hash_result_store.items():
            out[size] = []
            for val in vals:
                try:
                    ev = model.eval(val.raw)
                    out[size].append(ev.as_long() if hasattr(ev, "as_long") else int(ev))
                except (AttributeError, TypeError):
                    continue
        return out

    def find_concrete_keccak(self, data: S.BitVec) -> S.BitVec:
        digest = self.hasher(data.value.to_bytes(data.size() // 8, "big"))
        return S.symbol_factory.BitVecVal(int.from_bytes(digest, "big"), 256)

    def create_keccak(self, data: S.BitVec):
        length = data.size()
        func, inverse = self.get_function(length)
        if not data.symbolic:
            h = self.find_concrete_keccak(data)
            self.concrete_hashes[data] = h
            return h, S.And(func(data) == h, inverse(func(data)) == data)
        cond = self._create_condition(data)
        self.hash_result_store[length].append(func(data))
        return func(data), cond

    def _create_condition(self, func_input: S.BitVec) -> S.Bool:
        length = func_input.size()
        func, inv = self.get_function(length)
        if length not in self.interval_hook_for_size:
            self.interval_hook_for_size[length] = self._index_counter
            self._index_counter -= INTERVAL_DIFFERENCE
        lower = self.interval_hook_for_size[length] * PART
        upper = lower + PART
        cond = S.And(inv(func(func_input)) == func_input,
                     S.ULE(S.symbol_factory.BitVecVal(lower, 256), func(func_input)),
                     S.ULT(func(func_input), S.symbol_factory.BitVecVal(upper, 256)),
                     S.URem(func(func_input), S.symbol_factory.BitVecVal(64, 256)) == 0)
        concrete_cond = S.symbol_factory.Bool(False)
        for key, keccak in self.concrete_hashes.items():
            concrete_cond = S.Or(concrete_cond, S.And(func(func_input) == keccak, key == func_input))
        return S.And(inv(func(func_input)) == func_input, S.Or(cond, concrete_cond))


# ---------------------------------------------------------------------------
# symbolic world / transactions
# ---------------------------------------------------------------------------

ACTORS = (0xAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFE,      # CREATOR
          0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF,      # ATTACKER
          0xAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAA)      # SOMEGUY
CONTRACT = 0x0901D12EBE1B195E5AA8748E62BD7734AE19B51F
ADDR_MASK = (1 << 160) - 1


def bv(v: int, w: int = 256) -> S.BitVec:
    return S.symbol_factory.BitVecVal(v, w)


def _bitvec(x) -> S.BitVec:
    """``util.pop_bitvec`` (``laser/ethereum/util.py:67-88``)."""
    if isinstance(x, S.Bool):
        return S.If(x, bv(1), bv(0))
    if isinstance(x, int):
        return bv(x)
    return x


class Calldata:
    """``SymbolicCalldata`` (``calldata.py:207-232``)."""

    def __init__(self, tx_id: int):
        self.size = S.symbol_factory.BitVecSym("{}_calldatasize".format(tx_id), 256)
        self.array = S.Array("{}_calldata".format(tx_id), 256, 8)

    def load(self, item: S.BitVec) -> S.BitVec:
        return S.If(item < self.size, self.array[item], bv(0, 8))

    def word(self, offset) -> S.BitVec:
        """``get_word_at`` over the slice walk of ``BaseCalldata.__getitem__``:
        concrete offsets give constant indices, symbolic ones ``off + i``."""
        if isinstance(offset, int):
            parts = [self.load(bv(offset + i)) for i in range(32)]
        else:
            parts = [self.load(offset if i == 0 else offset + bv(i)) for i in range(32)]
        return S.Concat(parts)


class Storage:
    """``Storage`` (``account.py:18-62``): ``K(256, 256, 0)`` for an account
    created by the analysed creation transaction, ``Storage{addr}`` else."""

    def __init__(self, address: int, concrete: bool):
        self.array = S.K(256, 256, 0) if concrete else S.Array("Storage{}".format(address), 256, 256)

    def __getitem__(self, item: S.BitVec) -> S.BitVec:
        return self.array[item]

    def __setitem__(self, key: S.BitVec, value) -> None:
        self.array[key] = _bitvec(value)


class World:
    """Path constraints, balances, storage and the keccak manager of one
    symbolic execution path (``world_state.py``)."""

    def __init__(self, concrete_storage: bool = True):
        self.constraints: List[S.Bool] = []
        self.balance = S.Array("balance", 256, 256)          # world_state.py:33
        self.storage = Storage(CONTRACT, concrete_storage)
        self.kfm = KeccakFunctionManager()
        self.next_tx = 0
        # ground truth of the stream (recall labels): why the path became
        # infeasible, once it has (every later query of the world is UNSAT),
        # and whether any transaction wrote a WalletLibrary pending entry
        self.dead: Optional[str] = None
        self.pending_written = False
        self.allowance_written = False         # BECToken: any approve / increaseApproval

    def tx(self, creation: bool = False) -> "Tx":
        t = Tx(self, self.next_tx, creation)
        self.next_tx += 1
        return t

    def query(self, extra: Sequence[S.Bool] = ()) -> List[N.Node]:
        q = Query(c.raw for c in list(self.constraints) + list(extra))
        if extra:                              # a module's check: "open" unless labelled
            q.label = getattr(extra[-1], "check_label", "open")
        if self.dead:                          # the path itself is infeasible
            q.label = "unsat: " + self.dead
        return q

    def kill_path(self, why: str) -> None:
        """The path just became infeasible (by the stream's construction)."""
        if self.dead is None:
            self.dead = why


class Tx:
    """One message call (``transaction/symbolic.py:70-108``) or the contract
    creation (``:110-150``, caller = CREATOR)."""

    def __init__(self, world: World, tx_id: int, creation: bool):
        self.world = world
        self.id = tx_id
        self.caller = bv(ACTORS[0]) if creation else S.symbol_factory.BitVecSym(
            "sender_{}".format(tx_id), 256)
        self.callvalue = S.symbol_factory.BitVecSym("call_value{}".format(tx_id), 256)
        self.calldata = Calldata(tx_id)
        # initial_global_state_from_environment (transaction_models.py:121-133)
        bal = world.balance
        world.constraints.append(S.UGE(bal[self.caller], self.callvalue))
        bal[bv(CONTRACT)] = bal[bv(CONTRACT)] + self.callvalue
        bal[self.caller] = bal[self.caller] - self.callvalue
        # _setup_global_state_for_execution (symbolic.py:165-167)
        world.constraints.append(S.Or(*[self.caller == bv(a) for a in ACTORS]))

    # -- control flow -----------------------------------------------------------
    def jumpi(self, condition, taken: bool) -> None:
        """``jumpi_``: the true branch appends ``condi``, the false branch
        ``Not(condition)`` (a BitVec condition is compared with 0)."""
        if isinstance(condition, S.Bool):
            c = condition if taken else S.Not(condition)
        else:
            c = (condition != 0) if taken else (condition == 0)
        self.world.constraints.append(c)

    @staticmethod
    def iszero(x) -> S.BitVec:
        e = S.Not(x) if isinstance(x, S.Bool) else (x == 0)
        return S.If(e, bv(1), bv(0))

    def require(self, cond) -> None:
        """``require(c)``: ``c ISZERO PUSH tag JUMPI`` falls through on c."""
        self.jumpi(self.iszero(cond), taken=False)

    # -- ABI ----------------------------------------------------------------------
    def selector_expr(self) -> S.BitVec:
        return bv(0xFFFFFFFF) & S.UDiv(self.calldata.word(0), bv(1 << 224))

    def dispatch(self, selectors: Sequence[int], k: int) -> None:
        """The function dispatcher down to ``selectors[k]``."""
        self.jumpi(S.ULT(self.calldata.size, bv(4)), taken=False)
        sel = self.selector_expr()
        for j in range(k + 1):
            self.jumpi(bv(selectors[j]) == sel, taken=(j == k))

    def nonpayable(self) -> None:
        self.jumpi(self.iszero(self.callvalue), taken=True)

    def arg(self, i: int) -> S.BitVec:
        return self.calldata.word(4 + 32 * i)

    def arg_address(self, i: int) -> S.BitVec:
        return bv(ADDR_MASK) & self.arg(i)

    def sender(self) -> S.BitVec:
        return bv(ADDR_MASK) & self.caller

    # -- storage ------------------------------------------------------------------
    def sha3(self, data: S.BitVec) -> S.BitVec:
        h, cond = self.world.kfm.create_keccak(data)
        self.world.constraints.append(cond)
        return h

    def mapping(self, key: S.BitVec, slot: int) -> S.BitVec:
        """``keccak256(key . slot)``: the 64-byte memory of the Solidity
        mapping access, as one 512-bit Concat."""
        if not key.symbolic:
            return self.sha3(bv((key.value << 256) | slot, 512))
        return self.sha3(S.Concat(key, bv(slot)))

    def sload(self, idx) -> S.BitVec:
        return self.world.storage[_bitvec(idx)]

    def sstore(self, idx, value) -> None:
        self.world.storage[_bitvec(idx)] = value


# ---------------------------------------------------------------------------
# C1: suicide.sol -t 2
# ---------------------------------------------------------------------------

SUICIDE_FUNCS = [selector("kill(address)")]


def c1_queries(n: int = 64, seed: int = 0xC1) -> List[List[N.Node]]:
    """``Suicide.kill(address)`` over two transactions (``-t 2``): the
    is_possible checks of every JUMPI branch (``svm.py:257-262``) and the
    SWC-106 check ``addr == 0`` at SELFDESTRUCT."""
    rng = random.Random(seed)
    out: List[List[N.Node]] = []
    while len(out) < n:
        w = World(concrete_storage=True)
        for _ in range(1 + rng.randrange(2)):
            t = w.tx()
            if rng.randrange(3) == 0:                       # fallback: size < 4
                t.jumpi(S.ULT(t.calldata.size, bv(4)), taken=True)
                out.append(w.query())
                continue
            t.dispatch(SUICIDE_FUNCS, 0)
            out.append(w.query())
            addr = t.arg_address(0)
            hit = rng.randrange(2) == 0
            t.jumpi(S.Not(addr == bv(0)) if rng.randrange(2) else (addr == bv(0)), taken=hit)
            out.append(w.query())
    return out[:n]


# ---------------------------------------------------------------------------
# C3: BECToken.sol -t 3 integer-overflow checks
# ---------------------------------------------------------------------------

BEC_FUNCS = sorted(selector(s) for s in (
    "transfer(address,uint256)", "transferFrom(address,address,uint256)",
    "approve(address,uint256)", "batchTransfer(address[],uint256)",
    "increaseApproval(address,uint256)", "decreaseApproval(address,uint256)",
    "balanceOf(address)", "allowance(address,address)", "pause()", "unpause()"))
_BAL, _ALLOW, _OWNER_PAUSED, _TOTAL = 1, 2, 3, 0


# Ground-truth labels of the integer module's checks: a
# check the path itself rules out — SafeMath's own ``require`` on the same
# operands, appended before the query is posed — is UNSAT by construction and
# its label names that require; any other check is "open" (satisfiable or not:
# tests/planted.py looks for a model).  The label belongs to the check as
# created on its path (the wrapper object: hash-consing gives the same node to
# the same check expression on different paths, e.g. BECToken's multiply
# check after one or two receivers), kept as an attribute of that object
# (an id()-keyed map could hand a stale label to a later object at
# the same address, and popping it made a second query of one check "open");
# the query streams do not depend on it.


def _label(chk: S.Bool, label: str) -> S.Bool:
    chk.check_label = label
    return chk


class Query(list):
    """One query (a list of Bool DAG nodes, what get_model receives) with the
    generator's label: "unsat: <the require that rules it out>", "open" (a
    check nothing on the path rules out) or "path" (an is_possible query)."""

    label = "path"


def query_label(q: Sequence[N.Node]) -> str:
    return getattr(q, "label", "path")


def _when_not_paused(t: Tx) -> None:
    packed = t.sload(bv(_OWNER_PAUSED))                        # owner | paused << 160
    paused = bv(0xFF) & S.UDiv(packed, bv(1 << 160))
    t.require(t.iszero(paused))


def _bec_transfer(t: Tx, checks: List[S.Bool], from_arg: bool) -> None:
    k = BEC_FUNCS.index(selector("transferFrom(address,address,uint256)" if from_arg
                                 else "transfer(address,uint256)"))
    t.dispatch(BEC_FUNCS, k)
    t.nonpayable()
    _when_not_paused(t)
    frm = t.arg_address(0) if from_arg else t.sender()
    to = t.arg_address(1 if from_arg else 0)
    value = t.arg(2 if from_arg else 1)
    t.require(S.Not(to == bv(0)))
    slot_from = t.mapping(frm, _BAL)
    bal_from = t.sload(slot_from)
    t.require(S.And(S.UGT(value, bv(0)), S.Not(S.UGT(value, bal_from))))
    if from_arg:                                                # allowed[_from][msg.sender]
        allow = t.sload(t.sha3(S.Concat(t.sender(), t.mapping(frm, _ALLOW))))
        t.require(S.Not(S.UGT(value, allow)))
        if not t.world.allowance_written:
            # no allowance entry was ever stored (concrete storage: 0), and
            # value > 0 was required above
            t.world.kill_path("transferFrom before any approve: allowed[from][msg.sender] = 0 "
                              "< value")
    # SafeMath.sub: assert(b <= a); SUB annotated by the integer module
    t.require(S.Not(S.UGT(value, bal_from)))
    checks.append(_label(S.Not(S.BVSubNoUnderflow(bal_from, value, False)),
                         "unsat: SafeMath.sub require(value <= balances[from])"))
    t.sstore(slot_from, bal_from - value)
    slot_to = t.mapping(to, _BAL)
    bal_to = t.sload(slot_to)
    s = bal_to + value
    checks.append(_label(S.Not(S.BVAddNoOverflow(bal_to, value, False)),
                         "unsat: SafeMath.add require(balances[to] + value >= balances[to])"))
    t.require(S.Not(S.ULT(s, bal_to)))                         # SafeMath.add: assert(c >= a)
    t.sstore(slot_to, s)


def _bec_batch(t: Tx, checks: List[S.Bool], receivers: int) -> None:
    t.dispatch(BEC_FUNCS, BEC_FUNCS.index(selector("batchTransfer(address[],uint256)")))
    t.nonpayable()
    _when_not_paused(t)
    off = t.arg(0)                                              # ABI offset of _receivers
    cnt = t.calldata.word(off + bv(4))                          # _receivers.length
    value = t.arg(1)
    amount = cnt * value
    # the loop leaves after `receivers` iterations (i < cnt not taken), so
    # cnt <= receivers: one receiver cannot overflow cnt * value; two can
    # (the BEC bug: cnt = 2, value = 2^255)
    checks.append(_label(S.Not(S.BVMulNoOverflow(cnt, value, False)),
                         "open" if receivers >= 2 else
                         "unsat: loop exit (i < cnt not taken after 1 receiver) gives cnt <= 1"))
    t.require(S.And(S.UGT(cnt, bv(0)), S.Not(S.UGT(cnt, bv(20)))))
    slot_s = t.mapping(t.sender(), _BAL)
    bal_s = t.sload(slot_s)
    t.require(S.And(S.UGT(value, bv(0)), S.Not(S.ULT(bal_s, amount))))
    t.require(S.Not(S.UGT(amount, bal_s)))
    checks.append(_label(S.Not(S.BVSubNoUnderflow(bal_s, amount, False)),
                         "unsat: SafeMath.sub require(amount <= balances[sender])"))
    t.sstore(slot_s, bal_s - amount)
    for i in range(receivers):
        t.jumpi(S.ULT(bv(i), cnt), taken=True)                 # for (i < cnt)
        rcv = bv(ADDR_MASK) & t.calldata.word(off + bv(36 + 32 * i))
        slot_r = t.mapping(rcv, _BAL)
        bal_r = t.sload(slot_r)
        checks.append(_label(S.Not(S.BVAddNoOverflow(bal_r, value, False)),
                             "unsat: SafeMath.add require(balances[receiver] + value >= "
                             "balances[receiver])"))
        t.require(S.Not(S.ULT(bal_r + value, bal_r)))
        t.sstore(slot_r, bal_r + value)
    t.jumpi(S.ULT(bv(receivers), cnt), taken=False)


def _bec_approve(t: Tx, checks: List[S.Bool], increase: bool) -> None:
    name = "increaseApproval(address,uint256)" if increase else "approve(address,uint256)"
    t.dispatch(BEC_FUNCS, BEC_FUNCS.index(selector(name)))
    t.nonpayable()
    _when_not_paused(t)
    spender, value = t.arg_address(0), t.arg(1)
    outer = t.mapping(t.sender(), _ALLOW)
    slot = t.sha3(S.Concat(spender, outer))                     # allowed[owner][spender]
    t.world.allowance_written = True
    if increase:
        cur = t.sload(slot)
        checks.append(_label(S.Not(S.BVAddNoOverflow(cur, value, False)),
                             "unsat: SafeMath.add require(allowed + value >= allowed)"))
        t.require(S.Not(S.ULT(cur + value, cur)))
        t.sstore(slot, cur + value)
    else:
        t.sstore(slot, value)


def c3_queries(n: int = 256, seed: int = 0xC3) -> List[List[N.Node]]:
    """BECToken under ``-t 3``: up to three transactions after the creation
    transaction; every ADD/MUL/SUB the integer module annotates becomes one
    query ``path constraints + [Not(BV*NoOverflow(..))]`` at the end of the
    transaction (``integer.py:268-280``)."""
    rng = random.Random(seed)
    out: List[List[N.Node]] = []
    while len(out) < n:
        w = World(concrete_storage=True)
        c = w.tx(creation=True)                                 # constructor: totalSupply
        supply = bv(7000000000 * 10 ** 18)
        c.sstore(bv(_TOTAL), supply)
        c.sstore(c.mapping(bv(ACTORS[0]), _BAL), supply)
        c.sstore(bv(_OWNER_PAUSED), bv(ACTORS[0]))
        for _ in range(1 + rng.randrange(3)):
            t = w.tx()
            checks: List[S.Bool] = []
            kind = rng.randrange(6)
            if kind == 0:
                _bec_batch(t, checks, 1 + rng.randrange(2))
            elif kind in (1, 2):
                _bec_transfer(t, checks, from_arg=kind == 2)
            elif kind == 3:
                _bec_approve(t, checks, increase=True)
            elif kind == 4:
                _bec_approve(t, checks, increase=False)
            else:
                _bec_batch(t, checks, 1)
            for chk in checks:
                out.append(w.query([chk]))
    return out[:n]


# ---------------------------------------------------------------------------
# C4: WalletLibrary.sol + token.sol mapping / storage constraints
# ---------------------------------------------------------------------------

TOKEN_FUNCS = sorted(selector(s) for s in ("transfer(address,uint256)", "balanceOf(address)",
                                           "totalSupply()"))
WALLET_FUNCS = sorted(selector(s) for s in (
    "isOwner(address)", "confirm(bytes32)", "addOwner(address)", "execute(address,uint256,bytes)",
    "revoke(bytes32)", "changeOwner(address,address)", "kill(address)",
    "hasConfirmed(bytes32,address)", "initWallet(address[],uint256,uint256)"))
_W_REQUIRED, _W_NUMOWNERS, _W_OWNERS, _W_OWNERIDX, _W_PENDING = 0, 1, 2, 0x103, 0x104


def _token_transfer(t: Tx, checks: List[S.Bool]) -> None:
    """``token.sol`` ``transfer``: ``require(balances[msg.sender] - _value
    >= 0)`` (always true: the underflow is the finding), ``-=``, ``+=``."""
    t.dispatch(TOKEN_FUNCS, TOKEN_FUNCS.index(selector("transfer(address,uint256)")))
    to, value = t.arg_address(0), t.arg(1)
    slot_s = t.mapping(t.sender(), 0)
    bal_s = t.sload(slot_s)
    checks.append(S.Not(S.BVSubNoUnderflow(bal_s, value, False)))
    t.require(S.Not(S.ULT(bal_s - value, bv(0))))
    t.sstore(slot_s, t.sload(slot_s) - value)
    slot_t = t.mapping(to, 0)
    bal_t = t.sload(slot_t)
    checks.append(S.Not(S.BVAddNoOverflow(bal_t, value, False)))
    t.sstore(slot_t, bal_t + value)


def _wallet_owner_index(t: Tx, who: S.BitVec) -> S.BitVec:
    return t.sload(t.mapping(who, _W_OWNERIDX))                  # m_ownerIndex[uint(who)]


def _wallet_call(t: Tx, kind: int, checks: List[S.Bool], rng: random.Random) -> None:
    names = ["isOwner(address)", "confirm(bytes32)", "addOwner(address)",
             "execute(address,uint256,bytes)", "revoke(bytes32)", "kill(address)"]
    name = names[kind % len(names)]
    t.dispatch(WALLET_FUNCS, WALLET_FUNCS.index(selector(name)))
    if name == "isOwner(address)":
        t.jumpi(S.UGT(_wallet_owner_index(t, t.arg_address(0)), bv(0)), taken=rng.randrange(2) == 0)
        return
    t.nonpayable()
    if name in ("addOwner(address)", "kill(address)"):
        # onlymanyowners(keccak256(msg.data)): symbolic length -> forced 64
        t.world.constraints.append(t.calldata.size == bv(64))
        op = t.sha3(S.Concat(t.calldata.word(0), t.calldata.word(32)))
    elif name == "execute(address,uint256,bytes)":
        idx = _wallet_owner_index(t, t.sender())                  # onlyowner
        t.require(S.UGT(idx, bv(0)))
        value = t.arg(1)
        spent = t.sload(bv(0x105))
        # no transaction of the stream writes m_spentToday (slot 0x105): it is
        # 0 under the creation's storage, and 0 + value cannot overflow
        checks.append(_label(S.Not(S.BVAddNoOverflow(spent, value, False)),
                             "unsat: m_spentToday (slot 0x105) is never written, so "
                             "spent + value cannot overflow"))
        t.require(S.Not(S.UGT(spent + value, t.sload(bv(0x106)))))
        return
    else:
        op = t.arg(0)                                            # confirm / revoke(_h)
    # confirmAndCheck(_operation)
    idx = _wallet_owner_index(t, t.sender())
    t.require(S.Not(idx == bv(0)))
    pending = t.mapping(op, _W_PENDING)                         # m_pending[_operation]
    needed = t.sload(pending)
    zero = rng.randrange(2) == 0
    t.jumpi(needed == bv(0), taken=zero)
    # ground truth: a pending entry (a keccak slot of m_pending, a multiple of
    # 64 in its interval) holds 0 unless an earlier transaction wrote one
    if not zero and not t.world.pending_written:
        t.world.kill_path("m_pending[op].yetNeeded is 0 (no earlier transaction wrote a "
                          "pending entry), so the needed != 0 branch is infeasible")
    bit = t.sload(pending + bv(1))                              # ownersDone
    t.require(S.Not((bit & bv(1)) == bv(0)) if name == "revoke(bytes32)" else
              ((bit & bv(1)) == bv(0)))
    if name == "revoke(bytes32)":
        # pending + 1 is 1 mod 64: no keccak slot, no constant slot is ever
        # written there, so ownersDone is 0
        t.world.kill_path("ownersDone (slot pending + 1) is never written, so revoke's "
                          "require(ownersDone & 1) fails")
    chk = S.Not(S.BVSubNoUnderflow(needed, bv(1), False))
    checks.append(chk if zero else _label(chk, "unsat: the needed == 0 branch was not taken, "
                                                "so needed - 1 cannot underflow"))
    t.sstore(pending, needed - bv(1))
    t.world.pending_written = True


def c4_queries(n: int = 256, seed: int = 0xC4) -> List[List[N.Node]]:
    """``token.sol`` transfers and ``WalletLibrary`` owner / multi-sig paths
    over 1-3 transactions: every storage access is a keccak UF application
    over a 512-bit ``Concat(key, slot)`` read through a store chain, and
    every transaction carries its keccak conditions (the C4 shape)."""
    rng = random.Random(seed)
    out: List[List[N.Node]] = []
    while len(out) < n:
        w = World(concrete_storage=True)
        c = w.tx(creation=True)
        wallet = rng.randrange(2) == 0
        if wallet:                                              # initWallet([creator], 1, limit)
            c.sstore(bv(_W_NUMOWNERS), bv(1))
            c.sstore(bv(_W_OWNERS + 1), bv(ACTORS[0]))
            c.sstore(c.mapping(bv(ACTORS[0]), _W_OWNERIDX), bv(1))
            c.sstore(bv(_W_REQUIRED), bv(1))
        else:                                                   # constructor(_initialSupply)
            supply = c.arg(0)
            c.sstore(bv(1), supply)
            c.sstore(c.mapping(bv(ACTORS[0]), 0), supply)
        for _ in range(1 + rng.randrange(3)):
            t = w.tx()
            checks: List[S.Bool] = []
            if wallet:
                _wallet_call(t, rng.randrange(6), checks, rng)
            else:
                _token_transfer(t, checks)
            out.append(w.query())                              # is_possible of the new state
            for chk in checks:
                out.append(w.query([chk]))
    return out[:n]


# ---------------------------------------------------------------------------
# C5: every solidity_examples contract, batched.  Beyond the C1 / C3 / C4
# contracts above, the other nine (solidity_examples/*.sol) are restated
# here the same way: the dispatcher path of each function, its requires, and
# the query each detection module appends at the instruction it watches
# (analysis/module/modules/*.py).
# ---------------------------------------------------------------------------

def _env(t: Tx, name: str, w: int = 256) -> S.BitVec:
    """``GlobalState.new_bitvec``: ``{tx}_{name}`` (global_state.py:125-135)."""
    return S.symbol_factory.BitVecSym("{}_{}".format(t.id, name), w)


def _call(t: Tx, to: S.BitVec, checks: List[S.Bool], pc: int, checked: bool,
          value: Optional[S.BitVec] = None, not_attacker: Optional[str] = None) -> S.BitVec:
    """A CALL (``instructions.py:1920-2135``): ``retval_{pc}`` on the stack;
    the external-call module asks ``UGT(gas, 2300) ∧ to == ATTACKER``
    (``external_calls.py:79-84``), the unchecked-retval module
    ``retval == 1`` / ``retval == 0`` (``unchecked_retval.py:85-89``) when the
    result is not checked, the state-change module ``UGT(gas, 2300)`` with a
    positive value (``state_change_external_calls.py:47-62,196``).
    ``not_attacker``: why the target can never be the attacker (the
    external-call check is then UNSAT by construction: recall labels)."""
    gas = _env(t, "gas")
    ret = _env(t, "retval_%d" % pc)
    chk = S.And(S.UGT(gas, bv(2300)), to == bv(ACTORS[1]))
    checks.append(_label(chk, "unsat: " + not_attacker) if not_attacker else chk)
    if value is not None:
        checks.append(S.And(S.UGT(gas, bv(2300)), S.UGT(value, bv(0))))
    if checked:
        t.require(S.Not(ret == bv(0)))
    else:
        checks.append(ret == bv(1))
        checks.append(ret == bv(0))
    return ret


# deposits move msg.value out of the sender's ether (Tx: UGE(balance[caller],
# callvalue), then balance[caller] -= callvalue) into its balances[] entry, and
# withdrawals move it back: entry + ether stays at most the sender's ether
# before its first deposit, so entry + msg.value <= that, below 2^256
_DEPOSIT_NO_OVERFLOW = ("unsat: deposits move msg.value out of the sender's ether (bounded by "
                        "its balance), so balances[sender] + msg.value cannot overflow")


def _ether_thief(t: Tx, checks: List[S.Bool], amount: S.BitVec) -> None:
    """``ether_thief.py:60-72``: the attacker's balance after the transfer
    exceeds its starting balance, and the attacker sent the transaction."""
    bal = t.world.balance
    start = bal[bv(ACTORS[1])]
    bal[t.caller] = bal[t.caller] + amount
    checks.append(S.And(S.UGT(bal[bv(ACTORS[1])], start), t.caller == bv(ACTORS[1])))


CALLS_FUNCS = sorted(selector(x) for x in (
    "thisisfine()", "reentrancy()", "calluseraddress(address)", "callstoredaddress()",
    "setstoredaddress(address)", "fixed_address()", "stored_address()"))


def _calls_session(rng: random.Random, out: List[List[N.Node]]) -> None:
    """``calls.sol``: fixed / stored / user-supplied call targets."""
    w = World(concrete_storage=True)
    c = w.tx(creation=True)
    c.sstore(bv(0), c.arg_address(0))                           # fixed_address = addr
    stored = False                                              # slot 1 written yet
    for _ in range(1 + rng.randrange(2)):
        t = w.tx()
        checks: List[S.Bool] = []
        name = rng.choice(["thisisfine()", "reentrancy()", "calluseraddress(address)",
                           "callstoredaddress()", "setstoredaddress(address)"])
        t.dispatch(CALLS_FUNCS, CALLS_FUNCS.index(selector(name)))
        t.nonpayable()
        if name == "setstoredaddress(address)":
            t.sstore(bv(1), t.arg_address(0))
            stored = True
        else:
            if name == "calluseraddress(address)":
                to = t.arg_address(0)
            else:                                               # fixed / stored address
                to = bv(ADDR_MASK) & t.sload(bv(1 if name == "callstoredaddress()" else 0))
            never = None
            if name == "callstoredaddress()" and not stored:
                never = "stored_address (slot 1) was never set, so the call target is 0"
            _call(t, to, checks, 0x90 + len(name), checked=False, not_attacker=never)
            if name == "reentrancy()":
                t.sstore(bv(2), bv(0))                          # statevar = 0 after the call
        out.append(w.query())
        for chk in checks:
            out.append(w.query([chk]))


ETHERSTORE_FUNCS = sorted(selector(x) for x in (
    "depositFunds()", "withdrawFunds(uint256)", "withdrawalLimit()", "lastWithdrawTime(address)",
    "balances(address)"))


def _etherstore_session(rng: random.Random, out: List[List[N.Node]]) -> None:
    """``etherstore.sol``: deposit (``+= msg.value``, integer module) and
    withdraw (three requires, a call with value, then state changes)."""
    w = World(concrete_storage=True)
    c = w.tx(creation=True)
    c.sstore(bv(0), bv(10 ** 18))                               # withdrawalLimit = 1 ether
    withdrawn = False                                           # lastWithdrawTime written yet
    for _ in range(1 + rng.randrange(3)):
        t = w.tx()
        checks: List[S.Bool] = []
        if rng.randrange(2):
            t.dispatch(ETHERSTORE_FUNCS, ETHERSTORE_FUNCS.index(selector("depositFunds()")))
            slot = t.mapping(t.sender(), 2)
            cur = t.sload(slot)
            checks.append(_label(S.Not(S.BVAddNoOverflow(cur, t.callvalue, False)),
                                 _DEPOSIT_NO_OVERFLOW))
            t.sstore(slot, cur + t.callvalue)
        else:
            t.dispatch(ETHERSTORE_FUNCS, ETHERSTORE_FUNCS.index(selector("withdrawFunds(uint256)")))
            t.nonpayable()
            amt = t.arg(0)
            slot_b = t.mapping(t.sender(), 2)
            t.require(S.UGE(t.sload(slot_b), amt))
            t.require(S.ULE(amt, t.sload(bv(0))))
            now = _env(t, "timestamp")
            last = t.sload(t.mapping(t.sender(), 1))
            chk = S.Not(S.BVAddNoOverflow(last, bv(604800), False))
            checks.append(chk if withdrawn else _label(
                chk, "unsat: lastWithdrawTime[sender] is 0 until a withdrawal, so last + "
                     "604800 cannot overflow"))
            t.require(S.UGE(now, last + bv(604800)))
            _call(t, t.sender(), checks, 0x1F3, checked=True, value=amt)
            _ether_thief(t, checks, amt)
            bal = t.sload(slot_b)
            checks.append(S.Not(S.BVSubNoUnderflow(bal, amt, False)))
            t.sstore(slot_b, bal - amt)
            t.sstore(t.mapping(t.sender(), 1), now)
            withdrawn = True
        out.append(w.query())
        for chk in checks:
            out.append(w.query([chk]))


EXC_FUNCS = sorted(selector(x) for x in (
    "assert1()", "assert2()", "assert3(uint256)", "requireisfine(uint256)", "divisionby0(uint256)",
    "thisisfine(uint256)", "arrayaccess(uint256)", "thisisalsofind(uint256)"))


def _exceptions_session(rng: random.Random, out: List[List[N.Node]]) -> None:
    """``exceptions.sol``: the exceptions module asks whether each INVALID is
    reachable — the path to it (``exceptions.py:45-60``): ``input == 23``,
    a zero divisor (``ISZERO(input)`` before DIV), an index >= 8."""
    w = World(concrete_storage=True)
    w.tx(creation=True)
    t = w.tx()
    name = rng.choice(["assert3(uint256)", "requireisfine(uint256)", "divisionby0(uint256)",
                       "thisisfine(uint256)", "arrayaccess(uint256)", "thisisalsofind(uint256)"])
    t.dispatch(EXC_FUNCS, EXC_FUNCS.index(selector(name)))
    t.nonpayable()
    x = t.arg(0)
    if name == "assert3(uint256)":
        t.jumpi(S.Not(x == bv(23)), taken=False)                # to the INVALID
    elif name == "requireisfine(uint256)":
        t.require(S.Not(x == bv(23)))
    elif name == "divisionby0(uint256)":
        t.jumpi(t.iszero(x), taken=True)
    elif name == "thisisfine(uint256)":
        t.jumpi(S.UGT(x, bv(0)), taken=True)
        t.jumpi(t.iszero(x), taken=rng.randrange(2) == 0)
        t.sstore(bv(9), S.UDiv(bv(1), x))
    elif name == "arrayaccess(uint256)":
        t.jumpi(S.ULT(x, bv(8)), taken=False)                   # bounds check fails
    else:
        t.jumpi(S.ULT(x, bv(8)), taken=True)
        t.jumpi(S.ULT(x, bv(8)), taken=rng.randrange(2) == 0)
    out.append(w.query())


def _hashforether_session(rng: random.Random, out: List[List[N.Node]]) -> None:
    """``hashforether.sol``: ``require(uint32(msg.sender) == 0)`` then the
    whole balance to the sender (ether thief)."""
    funcs = sorted(selector(x) for x in ("withdrawWinnings()", "_sendWinnings()"))
    w = World(concrete_storage=True)
    w.tx(creation=True)
    for _ in range(1 + rng.randrange(2)):
        t = w.tx()
        checks: List[S.Bool] = []
        name = rng.choice(["withdrawWinnings()", "_sendWinnings()"])
        t.dispatch(funcs, funcs.index(selector(name)))
        t.nonpayable()
        if name == "withdrawWinnings()":
            t.require(S.Extract(31, 0, t.caller) == bv(0, 32))
        amount = w.balance[bv(CONTRACT)]
        _call(t, t.sender(), checks, 0x7A, checked=True, value=amount)
        _ether_thief(t, checks, amount)
        out.append(w.query())
        for chk in checks:
            out.append(w.query([chk]))


def _origin_session(rng: random.Random, out: List[List[N.Node]]) -> None:
    """``origin.sol``: ``require(tx.origin != owner)`` (origin = the sender,
    ``symbolic.py:98``), then ``if (newOwner != 0) owner = newOwner``."""
    funcs = sorted(selector(x) for x in ("transferOwnership(address)", "owner()"))
    w = World(concrete_storage=True)
    c = w.tx(creation=True)
    c.sstore(bv(0), c.sender())
    for _ in range(1 + rng.randrange(3)):
        t = w.tx()
        t.dispatch(funcs, funcs.index(selector("transferOwnership(address)")))
        t.nonpayable()
        owner = bv(ADDR_MASK) & t.sload(bv(0))
        t.require(S.Not(t.sender() == owner))
        out.append(w.query())
        new = t.arg_address(0)
        t.jumpi(S.Not(new == bv(0)), taken=rng.randrange(3) != 0)
        t.sstore(bv(0), new)
        out.append(w.query())


def _returnvalue_session(rng: random.Random, out: List[List[N.Node]]) -> None:
    """``returnvalue.sol``: the unchecked and the checked call."""
    funcs = sorted(selector(x) for x in ("callnotchecked()", "callchecked()", "callee()"))
    w = World(concrete_storage=True)
    c = w.tx(creation=True)
    c.sstore(bv(0), bv(0xE0F7E56E62B4267062172495D7506087205A4229))
    for _ in range(1 + rng.randrange(2)):
        t = w.tx()
        checks: List[S.Bool] = []
        name = rng.choice(["callnotchecked()", "callchecked()"])
        t.dispatch(funcs, funcs.index(selector(name)))
        t.nonpayable()
        _call(t, bv(ADDR_MASK) & t.sload(bv(0)), checks, 0x60 + len(name),
              checked=name == "callchecked()",
              not_attacker="the call target is the constant callee address (slot 0)")
        out.append(w.query())
        for chk in checks:
            out.append(w.query([chk]))


RUBIXI_FUNCS = sorted(selector(x) for x in (
    "dynamicPyramid()", "collectAllFees()", "collectFeesInEther(uint256)",
    "collectPercentOfFees(uint256)", "changeOwner(address)", "changeMultiplier(uint256)",
    "changeFeePercentage(uint256)", "currentMultiplier()", "totalParticipants()"))
_R_BAL, _R_FEES, _R_FEEPCT, _R_MULT, _R_ORDER, _R_CREATOR, _R_PARTS = 0, 1, 2, 3, 4, 5, 6


def _rubixi_session(rng: random.Random, out: List[List[N.Node]]) -> None:
    """``rubixi.sol``: the fallback's fee / payout arithmetic (MUL / DIV by
    100, ``+=`` checked by the integer module), the misnamed
    ``dynamicPyramid`` constructor and the ``onlyowner`` fee withdrawals."""
    w = World(concrete_storage=True)
    c = w.tx(creation=True)
    c.sstore(bv(_R_FEEPCT), bv(10))
    c.sstore(bv(_R_MULT), bv(300))
    creator = False                                             # slot 5 written yet
    for _ in range(1 + rng.randrange(3)):
        t = w.tx()
        checks: List[S.Bool] = []
        kind = rng.randrange(4)
        if kind == 0:                                           # fallback -> init()
            t.jumpi(S.ULT(t.calldata.size, bv(4)), taken=True)
            v = t.callvalue
            small = rng.randrange(2) == 0
            t.jumpi(S.ULT(v, bv(10 ** 18)), taken=small)
            fees = t.sload(bv(_R_FEES))
            if small:
                checks.append(S.Not(S.BVAddNoOverflow(fees, v, False)))
                t.sstore(bv(_R_FEES), fees + v)
            else:
                fee = t.sload(bv(_R_FEEPCT))
                big = rng.randrange(2) == 0
                t.jumpi(S.Not(S.ULT(v, bv(50 * 10 ** 18))), taken=big)
                if big:
                    fee = S.UDiv(fee, bv(2))
                mult = t.sload(bv(_R_MULT))
                checks.append(S.Not(S.BVMulNoOverflow(v, mult, False)))
                payout = S.UDiv(v * mult, bv(100))
                n_parts = t.sload(bv(_R_PARTS))
                checks.append(S.Not(S.BVAddNoOverflow(n_parts, bv(1), False)))
                t.sstore(bv(_R_PARTS), n_parts + bv(1))
                base = t.sha3(bv(_R_PARTS))
                t.sstore(base + bv(2) * n_parts + bv(1), payout)
                t.jumpi(n_parts + bv(1) == bv(10), taken=False)
                share = S.UDiv(v * (bv(100) - fee), bv(100))
                bal = t.sload(bv(_R_BAL))
                checks.append(S.Not(S.BVAddNoOverflow(bal, share, False)))
                t.sstore(bv(_R_BAL), bal + share)
                checks.append(S.Not(S.BVAddNoOverflow(fees, S.UDiv(v * fee, bv(100)), False)))
                first = t.sload(base + bv(2) * t.sload(bv(_R_ORDER)) + bv(1))
                t.jumpi(S.UGT(bal + share, first), taken=rng.randrange(2) == 0)
        elif kind == 1:
            t.dispatch(RUBIXI_FUNCS, RUBIXI_FUNCS.index(selector("dynamicPyramid()")))
            t.nonpayable()
            t.sstore(bv(_R_CREATOR), t.sender())
            creator = True
        else:
            name = "collectFeesInEther(uint256)" if kind == 2 else "collectPercentOfFees(uint256)"
            t.dispatch(RUBIXI_FUNCS, RUBIXI_FUNCS.index(selector(name)))
            t.nonpayable()
            t.jumpi(t.sender() == bv(ADDR_MASK) & t.sload(bv(_R_CREATOR)), taken=True)
            if not creator:
                w.kill_path("creator (slot 5) is 0 until dynamicPyramid() runs, so the "
                            "onlyowner test msg.sender == creator fails")
            fees = t.sload(bv(_R_FEES))
            arg = t.arg(0)
            if kind == 2:
                checks.append(S.Not(S.BVMulNoOverflow(arg, bv(10 ** 18), False)))
                amt = arg * bv(10 ** 18)
                t.jumpi(S.UGT(amt, fees), taken=False)
            else:
                t.require(S.And(S.UGT(fees, bv(0)), S.ULE(arg, bv(100))))
                amt = S.UDiv(fees, bv(100)) * arg
            t.require(S.UGT(fees, bv(0)))
            _call(t, bv(ADDR_MASK) & t.sload(bv(_R_CREATOR)), checks, 0x2C0 + kind, checked=True,
                  value=amt)
            _ether_thief(t, checks, amt)
            checks.append(S.Not(S.BVSubNoUnderflow(fees, amt, False)))
            t.sstore(bv(_R_FEES), fees - amt)
        out.append(w.query())
        for chk in checks:
            out.append(w.query([chk]))


def _timelock_session(rng: random.Random, out: List[List[N.Node]]) -> None:
    """``timelock.sol``: deposit (``now + 1 weeks``), increaseLockTime (the
    overflow the integer module finds), withdraw (``now > lockTime``: the
    predictable-variable module's ``timestamp`` dependence)."""
    funcs = sorted(selector(x) for x in ("deposit()", "increaseLockTime(uint256)", "withdraw()",
                                         "balances(address)", "lockTime(address)"))
    w = World(concrete_storage=True)
    w.tx(creation=True)
    locked = False                                              # a lockTime entry written yet
    for _ in range(1 + rng.randrange(3)):
        t = w.tx()
        checks: List[S.Bool] = []
        kind = rng.randrange(3)
        now = _env(t, "timestamp")
        slot_b, slot_l = t.mapping(t.sender(), 0), t.mapping(t.sender(), 1)
        if kind == 0:
            t.dispatch(funcs, funcs.index(selector("deposit()")))
            b = t.sload(slot_b)
            checks.append(_label(S.Not(S.BVAddNoOverflow(b, t.callvalue, False)),
                                 _DEPOSIT_NO_OVERFLOW))
            t.sstore(slot_b, b + t.callvalue)
            checks.append(S.Not(S.BVAddNoOverflow(now, bv(604800), False)))
            t.sstore(slot_l, now + bv(604800))
            locked = True
        elif kind == 1:
            t.dispatch(funcs, funcs.index(selector("increaseLockTime(uint256)")))
            t.nonpayable()
            cur = t.sload(slot_l)
            chk = S.Not(S.BVAddNoOverflow(cur, t.arg(0), False))
            checks.append(chk if locked else _label(
                chk, "unsat: lockTime[sender] is 0 until a deposit, so lockTime + "
                     "timeToIncrease cannot overflow"))
            t.sstore(slot_l, cur + t.arg(0))
        else:
            t.dispatch(funcs, funcs.index(selector("withdraw()")))
            t.nonpayable()
            t.require(S.UGT(t.sload(slot_b), bv(0)))
            t.require(S.UGT(now, t.sload(slot_l)))
            checks.append(S.ULT(t.sload(slot_l), now))          # predictable-variable check
            t.sstore(slot_b, bv(0))
            _call(t, t.sender(), checks, 0x1B0, checked=True, value=t.sload(slot_b))
        out.append(w.query())
        for chk in checks:
            out.append(w.query([chk]))


def _weakrandom_session(rng: random.Random, out: List[List[N.Node]]) -> None:
    """``weak_random.sol``: the payable fallback's ticket loop (``moneySent
    >= pricePerTicket && nextTicket < totalTickets``), and chooseWinner's
    ``coinbase % 50`` / ``sender % 50`` / ``difficulty`` hash."""
    w = World(concrete_storage=True)
    c = w.tx(creation=True)
    prize = 25 * 10 ** 17
    c.sstore(bv(0), bv(prize))
    c.sstore(bv(1), bv(50))
    c.sstore(bv(2), bv(prize // 50))
    c.sstore(bv(3), bv(1))
    sold = 0                                                    # nextTicket, concretely
    for _ in range(1 + rng.randrange(2)):
        t = w.tx()
        checks: List[S.Bool] = []
        t.jumpi(S.ULT(t.calldata.size, bv(4)), taken=True)
        money = t.callvalue
        for k in range(1 + rng.randrange(3)):
            price, nxt = t.sload(bv(2)), t.sload(bv(4))
            t.jumpi(S.And(S.UGE(money, price), S.ULT(nxt, t.sload(bv(1)))), taken=True)
            checks.append(_label(S.Not(S.BVAddNoOverflow(nxt, bv(1), False)),
                                 "unsat: nextTicket is the tickets sold so far (at most 6), "
                                 "so nextTicket + 1 cannot overflow"))
            t.sstore(bv(4), nxt + bv(1))
            sold += 1
            slot = t.sha3(S.Concat(nxt, bv(5)))
            t.sstore(slot, t.sender())
            t.sstore(slot + bv(1), t.sload(bv(3)))
            checks.append(S.Not(S.BVSubNoUnderflow(money, price, False)))
            money = money - price
        t.jumpi(S.And(S.UGE(money, t.sload(bv(2))), S.ULT(t.sload(bv(4)), t.sload(bv(1)))),
                taken=False)
        if rng.randrange(2):
            t.jumpi(t.sload(bv(4)) == t.sload(bv(1)), taken=True)
            if sold != 50:
                w.kill_path("nextTicket (%d tickets sold) is not totalTickets = 50, so "
                            "chooseWinner() is unreachable" % sold)
            cb = bv(ADDR_MASK) & _env(t, "coinbase")
            s1 = t.sload(t.sha3(S.Concat(S.URem(cb, t.sload(bv(1))), bv(5))))
            s2 = t.sload(t.sha3(S.Concat(S.URem(t.sender(), t.sload(bv(1))), bv(5))))
            h = t.sha3(S.Concat(bv(ADDR_MASK) & s1, bv(ADDR_MASK) & s2,
                                _env(t, "block_difficulty")))
            checks.append(S.ULT(S.URem(h, t.sload(bv(1))), bv(50)))
            t.sstore(bv(3), t.sload(bv(3)) + bv(1))
            t.sstore(bv(4), bv(0))
        t.jumpi(S.UGT(money, bv(0)), taken=rng.randrange(2) == 0)
        out.append(w.query())
        for chk in checks:
            out.append(w.query([chk]))


C5_EXTRA = {"calls": _calls_session, "etherstore": _etherstore_session,
            "exceptions": _exceptions_session, "hashforether": _hashforether_session,
            "origin": _origin_session, "returnvalue": _returnvalue_session,
            "rubixi": _rubixi_session, "timelock": _timelock_session,
            "weak_random": _weakrandom_session}


def contract_queries(name: str, n: int, seed: int) -> List[List[N.Node]]:
    """``n`` queries of one of the nine C5-only contracts (C5_EXTRA)."""
    rng = random.Random(seed)
    out: List[List[N.Node]] = []
    while len(out) < n:
        C5_EXTRA[name](rng, out)
    return out[:n]


# the thirteen solidity_examples contracts and their streams (C1 / C3 / C4
# for the four contracts those configs analyse)
C5_CONTRACTS = ("suicide", "BECToken", "token+WalletLibrary") + tuple(C5_EXTRA)


def c5_queries(n: int = 1024, seed: int = 0xC5) -> List[List[N.Node]]:
    """BASELINE config C5: every solidity_examples contract's query stream,
    batched — the C1 (suicide), C3 (BECToken) and C4 (token + WalletLibrary)
    stand-ins and the nine C5_EXTRA contracts, interleaved round-robin (one
    query per contract in turn) so any prefix mixes all thirteen."""
    per = -(-n // len(C5_CONTRACTS))
    streams = [c1_queries(per, seed ^ 0xC1), c3_queries(per, seed ^ 0xC3),
               c4_queries(per, seed ^ 0xC4)]
    streams += [contract_queries(name, per, seed ^ (0x100 + k))
                for k, name in enumerate(C5_EXTRA)]
    out: List[List[N.Node]] = []
    for i in range(per):
        for st in streams:
            if i < len(st):
                out.append(st[i])
    return out[:n]


def c3_overflow_queries(n: int = 64, seed: int = 0xC3) -> List[List[N.Node]]:
    """The C3 stream's open checks only — batchTransfer's ``cnt * value``
    after two receivers, each on its own path (the transactions before it
    differ) — for recall: the 64-query C3 prefix holds
    two.  Checks on a path an earlier transaction made infeasible are labelled
    unsat and left out, so each one here is SAT by construction (``cnt = 2``,
    ``value = 2^255`` makes ``amount`` 0).  Not a BASELINE configuration."""
    m = 32 * n
    while True:
        out = [q for q in c3_queries(m, seed) if query_label(q) == "open"]
        if len(out) >= n:
            return out[:n]
        m *= 2


WORKLOADS = {"c1": c1_queries, "c3": c3_queries, "c4": c4_queries, "c5": c5_queries,
             "c3o": c3_overflow_queries}


def queries(name: str, n: Optional[int] = None, seed: Optional[int] = None) -> List[List[N.Node]]:
    fn = WORKLOADS[name.lower()]
    kw = {}
    if n is not None:
        kw["n"] = n
    if seed is not None:
        kw["seed"] = seed
    return fn(**kw)
