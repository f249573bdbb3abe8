#!/bin/bash
# Round 3: smoke + PMC passes + SYRK split sweep
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"
true
true
bash tools/gpu/r3_pmc.sh || exit 1
cd "$R" && bash tools/gpu/r3_syrk3.sh || exit 1
