#!/bin/bash
# Stop a training job started by scripts/run_imagenet.sh (reference
# scripts/kill_python_procs.sh).  The reference runs `pkill python` on every
# node, which also kills unrelated jobs; this script signals only the
# launcher process groups recorded in $PIDFILE (torchrun and its ranks).
#
#   ./scripts/kill_python_procs.sh            # SIGTERM, then SIGKILL after 10 s
set -uo pipefail
PIDFILE=${PIDFILE:-/tmp/kfac_launch_${USER:-user}.pids}
if [[ ! -s "$PIDFILE" ]]; then
    echo "no launcher pids recorded in $PIDFILE" >&2
    exit 0
fi
stop_tree() {  # $1 = pid: signal the pid and all its descendants
    local sig=$2
    for c in $(pgrep -P "$1" 2>/dev/null); do stop_tree "$c" "$sig"; done
    kill "-$sig" "$1" 2>/dev/null || true
}
while read -r NODE PID; do
    if [[ "$NODE" == "$(hostname)" ]]; then
        echo "[$NODE] stopping launcher pid $PID"
        stop_tree "$PID" TERM
    else
        echo "[$NODE] stopping remote session of launcher pid $PID"
        # the local ssh client owns the remote session; closing it sends SIGHUP
        stop_tree "$PID" TERM
    fi
done < "$PIDFILE"
sleep 10
while read -r NODE PID; do
    if kill -0 "$PID" 2>/dev/null; then stop_tree "$PID" KILL; fi
done < "$PIDFILE"
rm -f "$PIDFILE"
