#!/bin/bash
# SQ counters for the AND chain under each experimental build (one pass each)
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
for lib in "$@"; do
  n=$(basename $lib .so)
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/pmc/$n -o run -- python3 tools/opbench.py --lib=$lib bvand > gpurun_out/pmc/$n.log 2>&1 || exit 1
done
