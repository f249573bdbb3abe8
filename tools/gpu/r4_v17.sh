#!/bin/bash
# Round 4: where the bench's extra refresh time goes (isolated real-factor
# refresh: 211 ms, profiles/refresh_replay_r4.json): eager bench, and the
# default bench with per-phase HIP-event timing.
set -o pipefail
O=gpurun_out/r4w; mkdir -p $O
timeout -k 10 400 python -u bench.py --steps 100 --warmup 10 --secondary-bf16 0 --baseline 0 --graphs 0 > $O/bench_eager.json 2> $O/b.err || exit 1
timeout -k 10 400 python -u bench.py --steps 100 --warmup 10 --secondary-bf16 0 --baseline 0 --phase-timing > $O/bench_phase.json 2>> $O/b.err || exit 1
for f in $O/bench_eager.json $O/bench_phase.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', d['value'], d['kind_ms'], d.get('eigen_refresh_ms'), d.get('phase_ms_per_step'))"; done
