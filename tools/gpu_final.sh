#!/bin/bash
# End-of-round evidence on one MI355X: the -m gpu suite, the default bench
# line (with its CPU leg), the rocprofv3 kernel trace / HBM / SQ passes of
# that configuration (tools/profile.sh), the search bench, and the C3 / C4
# eval-mode lines.  Each step has its own time limit; the first failure ends
# the script.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${1:-final}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; echo "gpu tests failed"; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -c 400 gpurun_out/${TAG}_bench.log
bash tools/profile.sh || { echo "profile failed"; exit 1; }
timeout -k 10 400 python -u tools/search_bench.py > gpurun_out/${TAG}_search.log 2>&1 || { tail -30 gpurun_out/${TAG}_search.log; exit 1; }
for W in c3 c4; do
  timeout -k 10 400 python -u bench.py --workload $W --no-cpu-baseline > gpurun_out/${TAG}_bench_$W.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_$W.log; exit 1; }
done
echo final-ok
