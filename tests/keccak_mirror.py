"""Test infrastructure: the reference's symbolic-hash encoding
(mythril/laser/ethereum/keccak_function_manager.py:24-149) as the workload
builders restate it (mythril_amd.workloads.KeccakFunctionManager), with a
pluggable hasher so the reference's keccak sat/unsat expectations
(tests/laser/keccak_tests.py) can be posed to the GPU search with the
product's GPU Keccak (mg_keccak256) hashing the concrete inputs."""

from mythril_amd.workloads import INTERVAL_DIFFERENCE, PART, TOTAL_PARTS  # noqa: F401
from mythril_amd.workloads import KeccakFunctionManager as KeccakManager  # noqa: F401
