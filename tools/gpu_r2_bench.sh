#!/bin/bash
# bench.py at the driver's settings, plus phase timing, plus an fp32 row.
set -o pipefail
mkdir -p gpurun_out/bench
O=gpurun_out/bench
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/b20.json 2>$O/b20.err || { tail -20 $O/b20.err; exit 1; }
cat $O/b20.json
timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --phase-timing > $O/b100.json 2>$O/b100.err || { tail -20 $O/b100.err; exit 1; }
cat $O/b100.json
