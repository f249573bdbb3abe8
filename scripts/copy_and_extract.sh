#!/bin/bash
# Copy a dataset archive to local storage on every node and extract it
# (reference scripts/copy_and_extract.sh).  Local NVMe keeps the data loader
# off the shared filesystem.
#
#   ./scripts/copy_and_extract.sh /shared/imagenet.tar /tmp/imagenet
#   NODEFILE=hosts ./scripts/copy_and_extract.sh ARCHIVE DEST
set -euo pipefail
if [[ $# -ne 2 ]]; then
    echo "usage: $0 ARCHIVE DEST_DIR" >&2
    exit 1
fi
ARCHIVE=$1
DEST=$2
if [[ -z "${NODEFILE:-}" && -n "${SLURM_NODELIST:-}" ]]; then
    NODEFILE=$(mktemp)
    scontrol show hostnames "$SLURM_NODELIST" > "$NODEFILE"
fi
if [[ -z "${NODEFILE:-}" ]]; then
    NODES=("$(hostname)")
else
    mapfile -t NODES < <(grep -v '^\s*$' "$NODEFILE")
fi
CMD="mkdir -p '$DEST' && cp '$ARCHIVE' '$DEST/' && tar -xf '$DEST/$(basename "$ARCHIVE")' -C '$DEST' && rm '$DEST/$(basename "$ARCHIVE")'"
for NODE in "${NODES[@]}"; do
    if [[ "$NODE" == "$(hostname)" ]]; then
        echo "[$NODE] $CMD"
        bash -c "$CMD" &
    else
        echo "[$NODE] $CMD"
        ssh "$NODE" "$CMD" &
    fi
done
wait
echo "done: $ARCHIVE -> $DEST on ${#NODES[@]} node(s)"
