#!/bin/bash
# JIT leaf layout without waterfall state on aligned waves: the -m gpu
# suite, then alternated A/B against MYTHGPU_GEN_JIT_FLAT=0 (same library:
# the knob only changes the compiled programs) on C4 and C2.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
TAG=${1:-r4fl}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; echo "gpu tests failed"; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
BENCH_ARGS="--workload c4" bash tools/gpu_ab.sh flat_c4 mythril_amd/lib/libmythgpu.so MYTHGPU_GEN_JIT_FLAT=0 || exit 1
BENCH_ARGS="--workload c3" bash tools/gpu_ab.sh flat_c3 mythril_amd/lib/libmythgpu.so MYTHGPU_GEN_JIT_FLAT=0 || exit 1
bash tools/gpu_ab.sh flat_c2 mythril_amd/lib/libmythgpu.so MYTHGPU_GEN_JIT_FLAT=0 || exit 1
echo flat-ok
