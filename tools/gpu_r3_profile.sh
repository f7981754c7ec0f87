#!/bin/bash
# Round-3 evidence run: rocprofv3 kernel trace + HBM counters + SQ counters of
# the default bench (tools/profile.sh), then the C3 / C4 eval-mode bench lines
# (with their CPU leg) and a kernel trace of each.  Stops at the first failure.
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export MYTHGPU_JIT_CACHE=/tmp/mg_jitcache
TAG=${1:-r3b}
bash tools/profile.sh || { echo "profile failed"; tail -20 gpurun_out/prof/*.log; exit 1; }
for W in c3 c4; do
  timeout -k 10 300 python3 -u bench.py --workload $W > gpurun_out/${TAG}_bench_$W.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_$W.log; exit 1; }
  mkdir -p gpurun_out/prof_$W
  ( cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$W/kt -o kt -- python3 bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$W/kt.log 2>&1 ) || { tail -20 gpurun_out/prof_$W/kt.log; exit 1; }
done
echo r3-profile-ok
