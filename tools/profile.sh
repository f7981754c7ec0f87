#!/bin/bash
# rocprofv3 evidence for the bench: kernel-trace stats, then separate PMC
# passes for HBM traffic (FETCH_SIZE, WRITE_SIZE) — one counter group per
# pass, as MI355X_MICROARCH.md's rocprofv3 section prescribes — and an SQ pass.
# The compiled-program images are assembled first, outside the profiler
# (bench.py --jit-build-only into $MYTHGPU_JIT_CACHE): a process the profiler
# has attached to the GPU never starts the assembler.
# usage: tools/profile.sh [bench args...]
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export MYTHGPU_JIT_CACHE=/tmp/mg_jitcache
ARGS="$@"
# a counter pass prints nothing for minutes: keep a heartbeat file moving
# (gpurun's watchdog), stopped when the script ends
( while true; do date >> gpurun_out/prof/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 300 python3 bench.py --jit-build-only $ARGS > gpurun_out/prof/prebuild.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --jit-build-only --dags 512 > gpurun_out/prof/prebuild512.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/kt -o kt -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline $ARGS > gpurun_out/prof/kt.log 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/fetch -o fetch -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline $ARGS > gpurun_out/prof/fetch.log 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/write -o write -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline $ARGS > gpurun_out/prof/write.log 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU --output-format csv -d gpurun_out/prof/sq -o sq -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --dags 512 > gpurun_out/prof/sq.log 2>&1 || exit 1
echo profile-ok
