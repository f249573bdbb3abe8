# eigh threaded-lane probe (tools/eigh_lanes_probe.py)
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
timeout -k 10 400 python3 -u "$R/tools/eigh_lanes_probe.py" > "$R/gpurun_out/eigh_lanes.jsonl" 2> "$R/gpurun_out/eigh_lanes.err"
