cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g6_tests.log 2>&1 || { tail -30 gpurun_out/g6_tests.log; exit 1; }
tail -1 gpurun_out/g6_tests.log
timeout -k 10 400 python -u tools/ab.py mythril_amd/lib/ab/libmythgpu_v5.so mythril_amd/lib/ab/libmythgpu_v6.so --ops bvadd --dags 512 --rounds 3 > gpurun_out/ab_gen6.log 2>&1 || { tail -20 gpurun_out/ab_gen6.log; exit 1; }
tail -4 gpurun_out/ab_gen6.log
for P in scratch4 scratch2 scratch8; do
MYTHRIL_GPU_LEAF_REMAT=$P timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/g6_bench_$P.log 2>&1 || { tail -20 gpurun_out/g6_bench_$P.log; exit 1; }
python -c "
import json; t=open('gpurun_out/g6_bench_$P.log').read(); d=json.loads(t[t.index('{'):])
print('$P value %.1f G  frac %.3f  kernel_ms %.1f' % (d['value']/1e9, d['roofline']['frac'], d['roofline']['kernel_ms']))"
done
