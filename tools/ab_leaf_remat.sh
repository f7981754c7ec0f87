#!/bin/bash
# A/B of the allocator's leaf eviction policy (ir.LEAF_REMAT) on the bench:
# time (two timed steps) and HBM traffic (separate FETCH_SIZE / WRITE_SIZE
# passes) per policy.
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/remat
for POL in "$@"; do
  MYTHRIL_GPU_LEAF_REMAT=$POL timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/remat/bench_$POL.log 2>&1 || { tail -5 gpurun_out/remat/bench_$POL.log; exit 1; }
  MYTHRIL_GPU_LEAF_REMAT=$POL timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/remat/fetch_$POL -o fetch -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/remat/fetch_$POL.log 2>&1 || exit 1
  MYTHRIL_GPU_LEAF_REMAT=$POL timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/remat/write_$POL -o write -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/remat/write_$POL.log 2>&1 || exit 1
  tail -1 gpurun_out/remat/bench_$POL.log | cut -c1-200
done
echo ab-ok
