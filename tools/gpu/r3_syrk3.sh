#!/bin/bash
# Round 3: SYRK split-count sweep per ResNet-50 factor shape (KFAC_SYRK_SPLITS overrides the heuristic)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3k3; mkdir -p $O
timeout -k 10 200 python3 -u tools/syrk_probe.py --json $O/auto.jsonl > $O/auto.log 2>&1 || { echo "auto rc=$?"; tail -5 $O/auto.log; exit 1; }
tail -1 $O/auto.log
for sp in 1 2 4 8 16 32; do
  KFAC_SYRK_SPLITS=$sp timeout -k 10 200 python3 -u tools/syrk_probe.py --json $O/sp$sp.jsonl > $O/sp$sp.log 2>&1 || { echo "sp$sp rc=$?"; tail -5 $O/sp$sp.log; exit 1; }
  tail -1 $O/sp$sp.log
done
