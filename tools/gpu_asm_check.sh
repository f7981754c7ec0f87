#!/bin/bash
# First MI355X run of the assembly interpreter: parity, per-op costs, bench A/B.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_model.py -x -v --timeout 120 --timeout-method thread > gpurun_out/asm_gpu_tests.log 2>&1 || { echo "gpu tests failed rc=$?"; exit 1; }
timeout -k 10 200 python -u tools/opbench.py > gpurun_out/asm_opbench.log 2>&1 || { echo "opbench failed"; exit 1; }
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/asm_bench.log 2>&1 || { echo "bench failed"; exit 1; }
MYTHGPU_KERNEL=cxx timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/cxx_bench.log 2>&1 || { echo "cxx bench failed"; exit 1; }
echo all-ok
