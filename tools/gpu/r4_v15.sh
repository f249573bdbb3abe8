#!/bin/bash
# Round 4: per-dispatch floor of dependent kernels (tools/launch_floor.cpp).
set -o pipefail
O=gpurun_out/r4u; mkdir -p $O
timeout -k 10 60 tools/bin/launch_floor 4000 > $O/launch_floor.json 2>&1 && \
timeout -k 10 60 tools/bin/launch_floor 4000 >> $O/launch_floor.json 2>&1
cat $O/launch_floor.json
