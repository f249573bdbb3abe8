#!/bin/bash
# Round 4: the bench's refresh on its real factors vs synthetic ones.
set -o pipefail
O=gpurun_out/r4v; mkdir -p $O
timeout -k 10 300 python -u tools/refresh_replay.py --steps 101 --reps 3 > $O/refresh_replay.json 2> $O/refresh_replay.err
cat $O/refresh_replay.json
