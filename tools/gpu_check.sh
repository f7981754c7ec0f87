#!/bin/bash
# Standard GPU round trip: parity tests, op microbenchmark, bench (no CPU leg).
# Each GPU step has its own time limit; the chain stops at the first failure.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
 && timeout -k 10 300 python -u tools/opbench.py ${OPBENCH_OPS:-} > gpurun_out/opbench.log 2>&1 \
 && timeout -k 10 600 python -u bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?
tail -2 gpurun_out/gpu_tests.log
echo "rc=$rc"
exit $rc
