"""Concrete hashes in reported transactions, batched on the GPU
(SURVEY.md §8f rank 3).

Reference: ``_replace_with_actual_sha`` (``mythril/analysis/solver.py:119-152``)
walks every 64-hex-digit window of each concrete transaction input that
contains ``hash_matcher`` (``"fffffff"``), finds the window's value among the
model's concrete hash outputs (``KeccakFunctionManager.get_concrete_hash_data``,
``keccak_function_manager.py:102-120``), evaluates the matching inverse
function at it and replaces the window with the real Keccak-256 of that
input (``find_concrete_keccak``, ``:43-57``).  The report shows the result,
so it must be byte-identical.

Here every Keccak the walk can need is computed in one batch first (one GPU
launch, ``mg_keccak256``, one lane per message): the windows of the original
inputs are scanned speculatively, their inverse inputs evaluated (cached) and
hashed together.  The reference's sequential walk then runs unchanged on the
cached digests — a replacement can create a window the first scan did not
see, and such a digest is computed on demand — so the output is the
reference's output.
"""

from __future__ import annotations

from typing import Callable, Dict, List, Optional, Sequence, Tuple

HASH_MATCHER = "fffffff"       # keccak_function_manager.py:20


def _as_int(v) -> int:
    return v.as_long() if hasattr(v, "as_long") else int(v)


def _gpu_keccak(msgs: Sequence[bytes]) -> List[bytes]:
    from .engine import get_engine
    return get_engine().keccak256(list(msgs))


def _windows(s: str, s_index: int):
    for i in range(s_index, len(s)):
        w = s[i:i + 64]
        if HASH_MATCHER in w and len(w) == 64:
            yield i, w


def replace_with_actual_sha(concrete_transactions: List[Dict[str, str]], model, keccak_manager,
                            code=None, symbol_factory=None,
                            keccak: Optional[Callable[[Sequence[bytes]], List[bytes]]] = None
                            ) -> None:
    """In-place drop-in for ``_replace_with_actual_sha(concrete_transactions,
    model, code)`` with the manager passed explicitly (the reference uses the
    module singleton).  ``symbol_factory`` builds the inverse's argument in
    the manager's expression layer (Mythril's ``laser.smt`` under Mythril);
    ``keccak`` hashes a batch of messages (default: the GPU)."""
    if symbol_factory is None:
        from .smt import symbol_factory
    keccak = keccak or _gpu_keccak
    concrete_hashes = keccak_manager.get_concrete_hash_data(model)
    inverses: Dict[Tuple[int, int], int] = {}

    def input_of(value: int) -> Optional[Tuple[int, int]]:
        found = None
        for size in concrete_hashes:                  # last matching size wins, as in the reference
            if value not in concrete_hashes[size]:
                continue
            key = (size, value)
            if key not in inverses:
                _, inverse = keccak_manager.store_function[size]
                inverses[key] = _as_int(model.eval(inverse(symbol_factory.BitVecVal(value, 256)).raw))
            found = (inverses[key], size)
        return found

    def message(inp: Tuple[int, int]) -> bytes:
        value, size = inp
        return (value % (1 << size)).to_bytes(size // 8, "big")

    def s_index_of(s: str) -> int:
        if code is not None and code.bytecode in s:
            return len(code.bytecode) + 2
        return 10

    # one batch for every digest the original inputs can need
    wanted: List[Tuple[int, int]] = []
    for tx in concrete_transactions:
        s = tx["input"]
        if HASH_MATCHER not in s:
            continue
        for _, w in _windows(s, s_index_of(s)):
            inp = input_of(int(w, 16))
            if inp is not None and inp not in wanted:
                wanted.append(inp)
    digests: Dict[Tuple[int, int], bytes] = {}
    if wanted:
        digests = dict(zip(wanted, keccak([message(i) for i in wanted])))

    # the reference's walk (solver.py:124-152) on the cached digests
    for tx in concrete_transactions:
        if HASH_MATCHER not in tx["input"]:
            continue
        s_index = s_index_of(tx["input"])
        for i in range(s_index, len(tx["input"])):
            data_slice = tx["input"][i:i + 64]
            if HASH_MATCHER not in data_slice or len(data_slice) != 64:
                continue
            inp = input_of(int(data_slice, 16))
            if inp is None:
                continue
            if inp not in digests:
                digests[inp] = keccak([message(inp)])[0]
            hex_keccak = digests[inp].hex().rjust(64, "0")
            tx["input"] = tx["input"][:s_index] + tx["input"][s_index:].replace(
                tx["input"][i:64 + i], hex_keccak)
