#!/bin/bash
# Round 4: rocprofv3 kernel statistics of the final default bench (fp32 run,
# SGD baseline and bf16 secondary included).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4p2; mkdir -p $O
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p8 -o p8 -- python3 bench.py --steps 20 --warmup 5 > $O/bench_prof.json 2> $O/prof.err || exit 1
S=$(find /tmp/p8 -name "*kernel_stats.csv" | head -1)
echo "stats: $S"
cp "$S" $O/kernel_stats_final_default.csv
head -25 $O/kernel_stats_final_default.csv | cut -c1-160
