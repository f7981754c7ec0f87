"""Test infrastructure: the reference's symbolic-hash encoding
(mythril/laser/ethereum/keccak_function_manager.py:24-149) rebuilt with the
z3-free expression mirror, so the reference's keccak sat/unsat expectations
(tests/laser/keccak_tests.py) can be posed to the GPU search.  Concrete hashes
come from the product's GPU Keccak (mg_keccak256)."""

from mythril_amd.smt import ULE, ULT, And, Function, Or, URem, symbol_factory

TOTAL_PARTS = 10 ** 40
PART = (2 ** 256 - 1) // TOTAL_PARTS
INTERVAL_DIFFERENCE = 10 ** 30


class KeccakManager:
    def __init__(self, hasher):
        self.hasher = hasher            # bytes -> 32-byte digest
        self.store_function = {}
        self.interval_hook_for_size = {}
        self._index_counter = TOTAL_PARTS - 34534
        self.concrete_hashes = {}
        self.hash_result_store = {}

    def get_function(self, length):
        if length not in self.store_function:
            self.store_function[length] = (Function("keccak256_{}".format(length), length, 256),
                                           Function("keccak256_{}-1".format(length), 256, length))
            self.hash_result_store[length] = []
        return self.store_function[length]

    def get_concrete_hash_data(self, model):
        """keccak_function_manager.py:102-120: the model's values of every
        symbolic hash created so far, per input size."""
        out = {}
        for size, vals in self.hash_result_store.items():
            out[size] = []
            for val in vals:
                try:
                    ev = model.eval(val.raw)
                    out[size].append(ev.as_long() if hasattr(ev, "as_long") else int(ev))
                except (AttributeError, TypeError):
                    continue
        return out

    def find_concrete_keccak(self, data):
        digest = self.hasher(data.value.to_bytes(data.size() // 8, "big"))
        return symbol_factory.BitVecVal(int.from_bytes(digest, "big"), 256)

    def create_keccak(self, data):
        length = data.size()
        func, inverse = self.get_function(length)
        if data.symbolic is False:
            h = self.find_concrete_keccak(data)
            self.concrete_hashes[data] = h
            return h, And(func(data) == h, inverse(func(data)) == data)
        cond = self._create_condition(data)
        self.hash_result_store[length].append(func(data))
        return func(data), cond

    def _create_condition(self, func_input):
        length = func_input.size()
        func, inv = self.get_function(length)
        if length not in self.interval_hook_for_size:
            self.interval_hook_for_size[length] = self._index_counter
            self._index_counter -= INTERVAL_DIFFERENCE
        index = self.interval_hook_for_size[length]
        lower = index * PART
        upper = lower + PART
        cond = And(inv(func(func_input)) == func_input,
                   ULE(symbol_factory.BitVecVal(lower, 256), func(func_input)),
                   ULT(func(func_input), symbol_factory.BitVecVal(upper, 256)),
                   URem(func(func_input), symbol_factory.BitVecVal(64, 256)) == 0)
        concrete_cond = symbol_factory.Bool(False)
        for key, keccak in self.concrete_hashes.items():
            concrete_cond = Or(concrete_cond, And(func(func_input) == keccak, key == func_input))
        return And(inv(func(func_input)) == func_input, Or(cond, concrete_cond))
