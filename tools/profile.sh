#!/bin/bash
# rocprofv3 evidence for the bench: kernel-trace stats, then separate PMC
# passes for HBM traffic (FETCH_SIZE, WRITE_SIZE) — one counter group per
# pass, as MI355X_MICROARCH.md's rocprofv3 section prescribes — and an SQ pass.
# The compiled-program images are assembled first, outside the profiler
# (bench.py --jit-build-only into $MYTHGPU_JIT_CACHE): a process the profiler
# has attached to the GPU never starts the assembler.
# usage: [PROF_TAG=c3] tools/profile.sh [bench args...]   (output in
# gpurun_out/prof[_<tag>]; every pass runs the bench's own configuration, so
# the SQ counters are keyed to the same kernel as the traffic: round 5)
cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
P=gpurun_out/prof${PROF_TAG:+_$PROF_TAG}
mkdir -p $P
export MYTHGPU_JIT_CACHE=/tmp/mg_jitcache
# under rocprofv3 every forked compile worker holds a GPU context too, and a
# pool's SIGTERM at shutdown can leave a counter pass hung in the profiler's
# signal handler (r4p6 WRITE_SIZE pass): profiled runs compile in-process
export MYTHGPU_BENCH_WORKERS=1
ARGS="$@"
# a counter pass prints nothing for minutes: keep a heartbeat file moving
# (gpurun's watchdog), stopped when the script ends
( while true; do date >> $P/heartbeat.txt; sleep 45; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
# (the prebuild runs outside the profiler: it may use a worker pool; the
# C2 image of the 11-slot layout takes ~290 s on one worker)
MYTHGPU_BENCH_WORKERS=16 timeout -k 10 600 python3 bench.py --jit-build-only $ARGS > $P/prebuild.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P/kt -o kt -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline $ARGS > $P/kt.log 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/fetch -o fetch -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline $ARGS > $P/fetch.log 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/write -o write -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline $ARGS > $P/write.log 2>&1 || exit 1
# SQ instruction / activity counters and GRBM_GUI_ACTIVE (the kernel's
# cycles, summed over the 8 XCDs) in one pass: 8 SQ + 1 GRBM counters
timeout -s KILL 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU GRBM_GUI_ACTIVE --output-format csv -d $P/sq -o sq -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline $ARGS > $P/sq.log 2>&1 || exit 1
echo profile-ok
