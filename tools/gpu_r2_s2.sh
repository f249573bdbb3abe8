#!/bin/bash
# Round 2, session 2: which path differs -- graph / StepGraphs / eager.
set -o pipefail
mkdir -p gpurun_out/r2s2
O=gpurun_out/r2s2
run() {
  local name=$1; shift
  timeout -k 10 120 python -u tools/graph_parity_probe.py "$@" > $O/$name.jsonl 2>$O/$name.err \
    || { echo PROBE_FAIL $name; tail -20 $O/$name.err; cat $O/$name.jsonl; exit 1; }
  echo "== $name"; cat $O/$name.jsonl
}
run det_graph_eager --a graph --b eager --deterministic
run det_step_eager --a step --b eager --deterministic
run nd_eager_eager --a eager --b eager
run nd_step_step --a step --b step
