#!/bin/bash
# Round-4 measurements beyond the default line: C3 / C4 eval-mode bench lines
# (fused calldata words), the compiled-code probe of the search path, the
# superset-memo census, the search bench.  Each GPU step has its own limit;
# the chain stops at the first failure.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
# long fixtures (oracle runs over every bench unit, image assembly) print
# nothing for minutes: keep a heartbeat file moving for gpurun's watchdog
( while true; do date >> gpurun_out/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
TAG=${1:-r4m}
for W in c3 c4; do
  for P in ${REMAT_POLICIES:-scratch2}; do
    MYTHRIL_GPU_LEAF_REMAT=$P timeout -k 10 400 python -u bench.py --workload $W --no-cpu-baseline > gpurun_out/${TAG}_bench_${W}_$P.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_${W}_$P.log; exit 1; }
    tail -c 300 gpurun_out/${TAG}_bench_${W}_$P.log
  done
done
timeout -k 10 300 python -u tools/search_jit_probe.py > gpurun_out/${TAG}_search_jit.log 2>&1 || { tail -20 gpurun_out/${TAG}_search_jit.log; exit 1; }
timeout -k 10 400 python -u tools/superset_census.py > gpurun_out/${TAG}_superset.log 2>&1 || { tail -20 gpurun_out/${TAG}_superset.log; exit 1; }
tail -2 gpurun_out/${TAG}_superset.log
timeout -k 10 400 python -u tools/search_bench.py --skip-corpus > gpurun_out/${TAG}_search.log 2>&1 || { tail -20 gpurun_out/${TAG}_search.log; exit 1; }
echo measure-ok
