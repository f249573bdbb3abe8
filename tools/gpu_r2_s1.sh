#!/bin/bash
# Round 2, session 1: split-K determinism tests + graph-vs-eager bisect.
set -o pipefail
mkdir -p gpurun_out/r2s1
O=gpurun_out/r2s1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_kernels_gpu.py > $O/kern.log 2>&1 || { echo KERN_FAIL; tail -30 $O/kern.log; exit 1; }
tail -3 $O/kern.log
run() {  # name, env..., -- args
  local name=$1; shift
  timeout -k 10 120 env "$@" python -u tools/graph_parity_probe.py $PROBE_ARGS > $O/probe_$name.jsonl 2>$O/probe_$name.err \
    || { echo PROBE_FAIL $name; tail -20 $O/probe_$name.err; cat $O/probe_$name.jsonl; exit 1; }
  echo "== $name"; cat $O/probe_$name.jsonl
}
PROBE_ARGS="--method eigen" run eigen KFAC_X=1
PROBE_ARGS="--method eigen --deterministic" run eigen_det KFAC_X=1
PROBE_ARGS="--method inverse" run inverse KFAC_X=1
PROBE_ARGS="--method eigen" run eigen_nofs KFAC_FACTOR_STREAM=0
PROBE_ARGS="--method eigen" run eigen_nostepgraphs KFAC_GRAPHS=0
