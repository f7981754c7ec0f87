cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/remat_c2
for R in 1 2; do for P in scratch scratch2; do
  L=gpurun_out/remat_c2/${P}_$R.log
  MYTHRIL_GPU_LEAF_REMAT=$P timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $L 2>&1 || { tail -20 $L; exit 1; }
  python -c "
import json; t=open('$L').read(); d=json.loads(t[t.index('{\"metric'):])
print('$P $R %.1f G frac %.4f' % (d['value']/1e9, d['roofline']['frac']))"
done; done
