#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ from the reference's own
test data (run in the build container, where /root/reference exists; the GPU
box only reads the committed JSON).

Nothing from the reference is imported or executed: the VMTest JSON files are
read as data and the pytest parameter tables of
``tests/instructions/{shl,shr,sar}_test.py`` are read with ``ast`` (literal
tuples only).

Outputs
* ``vmtests.json``  — straight-line VMTest programs from ``vmArithmeticTest``
  and ``vmBitwiseLogicOperation`` (PUSH/DUP/SWAP/POP + arithmetic/bitwise ops +
  SSTORE), with their expected post-storage (the ethereum/tests filler's
  answer).  ``tests/evm_mini.py`` lowers them to DAGs the way
  ``mythril/laser/ethereum/instructions.py:330-758`` does.
* ``eip145.json``   — (value, shift, expected) vectors for SHL/SHR/SAR.
* ``keccak_kat.json`` — Keccak-256 of the zero strings hashed by
  ``vmSha3Test`` (SHA3 over untouched memory) with the expected digest.
"""

import ast
import glob
import json
import os
import sys

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

SUPPORTED = {
    0x00: "STOP", 0x01: "ADD", 0x02: "MUL", 0x03: "SUB", 0x04: "DIV", 0x05: "SDIV",
    0x06: "MOD", 0x07: "SMOD", 0x08: "ADDMOD", 0x09: "MULMOD", 0x0B: "SIGNEXTEND",
    0x10: "LT", 0x11: "GT", 0x12: "SLT", 0x13: "SGT", 0x14: "EQ", 0x15: "ISZERO",
    0x16: "AND", 0x17: "OR", 0x18: "XOR", 0x19: "NOT", 0x1A: "BYTE", 0x1B: "SHL",
    0x1C: "SHR", 0x1D: "SAR", 0x50: "POP", 0x55: "SSTORE",
}


def straight_line(code: bytes) -> bool:
    i = 0
    while i < len(code):
        op = code[i]
        if 0x60 <= op <= 0x7F:
            i += op - 0x5F + 1
            continue
        if 0x80 <= op <= 0x9F:
            i += 1
            continue
        if op not in SUPPORTED:
            return False
        i += 1
    return True


def vmtests():
    out = []
    for suite in ("vmArithmeticTest", "vmBitwiseLogicOperation"):
        for f in sorted(glob.glob(os.path.join(REF, "tests/laser/evm_testsuite/VMTests", suite, "*.json"))):
            with open(f) as fh:
                d = json.load(fh)
            for name, t in d.items():
                post = t.get("post")
                if not post:
                    continue
                code = bytes.fromhex(t["exec"]["code"][2:])
                if not straight_line(code):
                    continue
                addr = t["exec"]["address"]
                pre_storage = t["pre"].get(addr, {}).get("storage", {})
                if pre_storage:
                    continue
                out.append({
                    "suite": suite, "name": name, "code": code.hex(),
                    "storage": {k: v for k, v in post[addr]["storage"].items()},
                })
    return out


def eip145():
    out = []
    for op in ("shl", "shr", "sar"):
        path = os.path.join(REF, "tests/instructions/%s_test.py" % op)
        with open(path) as fh:
            tree = ast.parse(fh.read())
        for node in ast.walk(tree):
            if isinstance(node, ast.Call) and getattr(node.func, "attr", "") == "parametrize":
                if len(node.args) >= 2 and isinstance(node.args[0], ast.Constant) \
                        and node.args[0].value.replace(" ", "").startswith("val1,val2,expected"):
                    for tup in ast.literal_eval(node.args[1]):
                        out.append({"op": op, "value": tup[0], "shift": tup[1], "expected": tup[2]})
    return out


def keccak_kat():
    out = []
    for f in sorted(glob.glob(os.path.join(REF, "tests/laser/evm_testsuite/VMTests/vmSha3Test/*.json"))):
        with open(f) as fh:
            d = json.load(fh)
        for name, t in d.items():
            post = t.get("post")
            if not post:
                continue
            code = bytes.fromhex(t["exec"]["code"][2:])
            # PUSHa len PUSHb off SHA3 PUSH1 0 SSTORE
            stack, i = [], 0
            ok = True
            while i < len(code):
                op = code[i]
                if 0x60 <= op <= 0x7F:
                    n = op - 0x5F
                    stack.append(int.from_bytes(code[i + 1:i + 1 + n], "big"))
                    i += n + 1
                elif op == 0x20:
                    off, length = stack.pop(), stack.pop()
                    stack.append(("sha3", length))
                    i += 1
                elif op == 0x55:
                    i += 1
                    break
                else:
                    ok = False
                    break
            if not ok or not stack or not isinstance(stack[0], tuple):
                continue
            length = stack[0][1]
            digest = list(post.values())[0]["storage"]["0x00"]
            out.append({"name": name, "msg_hex": "00" * length, "digest": digest})
    return out


def main():
    if not os.path.isdir(REF):
        sys.exit("reference tree not present; fixtures are already committed")
    for fname, data in (("vmtests.json", vmtests()), ("eip145.json", eip145()),
                        ("keccak_kat.json", keccak_kat())):
        with open(os.path.join(HERE, fname), "w") as fh:
            json.dump(data, fh, indent=1, sort_keys=True)
        print(fname, len(data))


if __name__ == "__main__":
    main()
