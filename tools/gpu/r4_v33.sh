#!/bin/bash
# Round 4: the whole GPU suite and smoke on the final tree.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4q2; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread tests > $O/pytest_gpu_all.log 2>&1
echo "suite rc=$?"; tail -2 $O/pytest_gpu_all.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
