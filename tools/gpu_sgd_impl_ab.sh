# torch.optim.SGD fused vs foreach in the bench (alternating, same box)
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
for rep in 1 2; do
 for v in foreach fused; do
  timeout -k 10 400 python3 bench.py --steps 100 --warmup 10 --sgd-impl $v > gpurun_out/sgd_$v.json 2> gpurun_out/sgd_$v.err || { tail -5 gpurun_out/sgd_$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/sgd_$v.json').read().strip().splitlines()[-1]);print('$v', $rep, d['value'], d['ms_per_step'], d['kind_ms'], d.get('sgd_ms_per_step'), d.get('kfac_overhead_ms'))"
 done
done
