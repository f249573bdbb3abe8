#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/bj
O=gpurun_out/bj
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "block_jacobi or warm_start or eigh" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u tools/bj_probe.py --sizes 1152,2304,4608 --syevd 0 --configs 1:1e-6:4e-6:1,1:1e-5:4e-6:1 > $O/probe3.jsonl 2>$O/probe3.err || { tail -30 $O/probe3.err; cat $O/probe3.jsonl; exit 1; }
cat $O/probe3.jsonl
for cfg in "KFAC_BJ_TOL=1e-6" "KFAC_BJ_TOL=1e-5"; do
  env $cfg timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --baseline 0 > $O/bench_$cfg.json 2>$O/bench_$cfg.err || { tail -20 $O/bench_$cfg.err; exit 1; }
  echo "== $cfg"; cat $O/bench_$cfg.json
done
