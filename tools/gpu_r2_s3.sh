#!/bin/bash
set -o pipefail
O=gpurun_out/s3; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --baseline 0 --kfac-inv-method > $O/bench_inv.json 2>$O/bench_inv.err || { tail -20 $O/bench_inv.err; exit 1; }
cat $O/bench_inv.json
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2>$O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
