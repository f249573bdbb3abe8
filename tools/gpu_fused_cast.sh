# fused weight cast: GPU tests, then SGD + K-FAC bench A/B (alternating)
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fused_cast.py tests/test_graphs.py -m gpu > gpurun_out/fc_tests.log 2>&1; rc=$?; tail -3 gpurun_out/fc_tests.log; [ $rc = 0 ] || exit $rc
for rep in 1 2; do
 for v in 0 1; do
  timeout -k 10 400 python3 bench.py --steps 100 --warmup 10 --fused-weight-cast $v > gpurun_out/fc_$v.json 2> gpurun_out/fc_$v.err || { tail -5 gpurun_out/fc_$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/fc_$v.json').read().strip().splitlines()[-1]);print('fused', $v, $rep, d['value'], d['ms_per_step'], d['kind_ms'], d.get('sgd_ms_per_step'), d.get('kfac_overhead_ms'))"
 done
done
