# whole-step HIP graph probe (tools/graph_step_probe.py)
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
timeout -k 10 300 python3 -u "$R/tools/graph_step_probe.py" > "$R/gpurun_out/graph_probe.jsonl" 2> "$R/gpurun_out/graph_probe.err"
