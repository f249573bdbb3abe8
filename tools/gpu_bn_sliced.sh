# sliced two-launch BN path: GPU tests, then bench A/B (KFAC_BN_SLICED=0/1)
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bnact_gpu.py tests/test_graphs.py -m gpu > gpurun_out/bn_tests.log 2>&1; rc=$?; tail -2 gpurun_out/bn_tests.log; [ $rc = 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/bn_tests.log | head -20; exit $rc; }
for rep in 1 2; do
 for v in 0 1; do
  KFAC_BN_SLICED=$v timeout -k 10 400 python3 bench.py --steps 100 --warmup 10 > gpurun_out/bns_$v.json 2> gpurun_out/bns_$v.err || { tail -5 gpurun_out/bns_$v.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/bns_$v.json').read().strip().splitlines()[-1]);print('sliced', $v, $rep, d['value'], d['ms_per_step'], d['kind_ms'], d.get('sgd_ms_per_step'), d.get('kfac_overhead_ms'))"
 done
done
