set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
timeout -k 10 500 python3 "$R/tools/bench_eigh.py" > "$R/gpurun_out/eigh_sizes2.jsonl" 2> "$R/gpurun_out/eigh_sizes2.err"
