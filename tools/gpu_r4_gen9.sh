#!/bin/bash
# Generator v9 (one-multiply mixer) on one box: the -m gpu suite, then an
# alternated A/B against the v8 build (mythril_amd/lib/ab/libmythgpu_gen8.so,
# knob MYTHGPU_GEN_MIX=8) on C4 and C2.  Each GPU step has its own limit;
# the chain stops at the first failure.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
( while true; do date >> gpurun_out/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
TAG=${1:-r4v9}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; echo "gpu tests failed"; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
BENCH_ARGS="--workload c4" bash tools/gpu_ab.sh gen9_c4 mythril_amd/lib/ab/libmythgpu_gen8.so MYTHGPU_GEN_MIX=8 || exit 1
BENCH_ARGS="--workload c3" bash tools/gpu_ab.sh gen9_c3 mythril_amd/lib/ab/libmythgpu_gen8.so MYTHGPU_GEN_MIX=8 || exit 1
bash tools/gpu_ab.sh gen9_c2 mythril_amd/lib/ab/libmythgpu_gen8.so MYTHGPU_GEN_MIX=8 || exit 1
echo gen9-ok
