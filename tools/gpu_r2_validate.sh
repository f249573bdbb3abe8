# full GPU suite, stem SYRK timing, default bench
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out; cd $R
timeout -k 10 150 python3 -u tools/syrk_stem_time.py > gpurun_out/syrk_stem.json 2>&1 || { cat gpurun_out/syrk_stem.json; exit 1; }
cat gpurun_out/syrk_stem.json
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head; exit $rc; }
timeout -k 10 400 python3 bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -5 gpurun_out/bench_default.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/bench_default.json').read().strip().splitlines()[-1]);print({k:d.get(k) for k in ('value','ms_per_step','kind_ms','inverse_ms_each','sgd_ms_per_step','kfac_overhead_ms','vs_baseline')})"
