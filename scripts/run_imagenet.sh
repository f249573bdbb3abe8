#!/bin/bash
# Launch the ImageNet K-FAC example on one or more MI355X nodes
# (reference scripts/run_imagenet.sh).
#
#   ./scripts/run_imagenet.sh [training args...]          # this node, all GPUs
#   NODEFILE=hosts ./scripts/run_imagenet.sh --epochs 55  # multi-node over ssh
#   sbatch -N 4 scripts/run_imagenet.sh                   # Slurm (nodelist inferred)
#
# One process per GPU (torchrun --nproc-per-node = number of visible GPUs),
# RCCL over xGMI inside a node.  Environment knobs:
#   SCRIPT     training script (default examples/torch_imagenet_resnet.py)
#   NPROC      processes per node (default: number of GPUs from rocm-smi)
#   RDZV_PORT  rendezvous port for multi-node runs (default 29400)
#   PRELOAD    shell snippet run before the launcher (env activation, ...)
# Every launched torchrun PID is written to $PIDFILE (default
# /tmp/kfac_launch_$USER.pids) so scripts/kill_python_procs.sh can stop
# exactly these processes.
set -euo pipefail
cd "$(dirname "$0")/.."

SCRIPT=${SCRIPT:-examples/torch_imagenet_resnet.py}
PRELOAD=${PRELOAD:-"export OMP_NUM_THREADS=8 HSA_ENABLE_IPC_MODE_LEGACY=0 ;"}
RDZV_PORT=${RDZV_PORT:-29400}
PIDFILE=${PIDFILE:-/tmp/kfac_launch_${USER:-user}.pids}

if [[ -z "${NPROC:-}" ]]; then
    NPROC=$(python -c 'import torch; print(max(torch.cuda.device_count(), 1))')
fi

if [[ -z "${NODEFILE:-}" ]]; then
    if [[ -n "${SLURM_NODELIST:-}" ]]; then
        NODEFILE=$(mktemp)
        scontrol show hostnames "$SLURM_NODELIST" > "$NODEFILE"
    elif [[ -n "${COBALT_NODEFILE:-}" ]]; then
        NODEFILE=$COBALT_NODEFILE
    fi
fi
if [[ -z "${NODEFILE:-}" ]]; then
    NODES=("$(hostname)")
else
    mapfile -t NODES < <(grep -v '^\s*$' "$NODEFILE")
fi
NNODES=${#NODES[@]}

LAUNCHER="python -m torch.distributed.run --nnodes=$NNODES --nproc-per-node=$NPROC --max-restarts=0"
if [[ "$NNODES" -eq 1 ]]; then
    LAUNCHER+=" --standalone --local-addr 127.0.0.1"
else
    LAUNCHER+=" --rdzv-backend=c10d --rdzv-endpoint=${NODES[0]}:$RDZV_PORT --rdzv-id=kfac_$$"
fi
ARGS=$(printf ' %q' "$@")
FULL_CMD="$PRELOAD $LAUNCHER $SCRIPT$ARGS"
echo "Training command: $FULL_CMD"

: > "$PIDFILE"
for NODE in "${NODES[@]}"; do
    if [[ "$NODE" == "$(hostname)" || "$NNODES" -eq 1 ]]; then
        echo "Launching on local node $NODE"
        bash -c "$FULL_CMD" &
    else
        echo "Launching on remote node $NODE"
        ssh "$NODE" "cd $PWD && $FULL_CMD" &
    fi
    echo "$NODE $!" >> "$PIDFILE"
done
wait
