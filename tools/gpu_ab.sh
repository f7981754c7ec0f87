#!/bin/bash
# GPU A/B round: the -m gpu suite on the in-tree library, then tools/ab.py
# over every mythril_amd/lib/ab/*.so (base first), then the default bench.
# usage: tools/gpu_ab.sh <tag>
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${1:-ab}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
LIBS="mythril_amd/lib/ab/libmythgpu_base.so $(ls mythril_amd/lib/ab/*.so | grep -v _base.so)"
timeout -k 10 500 python -u tools/ab.py $LIBS --ops bvadd,bvudiv,bvurem --dags 512 --rounds 3 > gpurun_out/${TAG}_ab.log 2>&1 || { tail -20 gpurun_out/${TAG}_ab.log; exit 1; }
grep -E "^(corpus|bvudiv|bvurem)" gpurun_out/${TAG}_ab.log
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
python -c "
import json; t=open('gpurun_out/${TAG}_bench.log').read(); d=json.loads(t[t.index('{'):])
print('value %.1f G  frac %.3f  kernel_ms %.1f' % (d['value']/1e9, d['roofline']['frac'], d['roofline']['kernel_ms']))"
