#!/bin/bash
# Probes behind the spill-placement and VALU-ceiling decisions: VALU issue
# rates with the in-kernel clock (tools/valu_rate.hip) and the spill probe
# (tools/spill_probe.hip) with separate FETCH_SIZE / WRITE_SIZE passes.
# Binaries are built beforehand on the CPU side (hipcc cross-compiles).
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
timeout -k 10 120 tools/valu_rate > gpurun_out/probe/valu_rate.log 2>&1 || { tail gpurun_out/probe/valu_rate.log; exit 1; }
timeout -k 10 200 tools/spill_probe 8 > gpurun_out/probe/spill.log 2>&1 || { tail gpurun_out/probe/spill.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/probe/fetch -o fetch -- tools/spill_probe 8 > gpurun_out/probe/fetch.log 2>&1 || { tail gpurun_out/probe/fetch.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/probe/write -o write -- tools/spill_probe 8 > gpurun_out/probe/write.log 2>&1 || { tail gpurun_out/probe/write.log; exit 1; }
echo probe-ok
