#!/bin/bash
# Round 3: graph replays with no eager work in between (sequential twin) vs interleaved
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3bn3; mkdir -p $O
timeout -k 10 200 python -u tools/graph_nan_probe.py --steps 6 --image 224 --batch 32 --fused-sgd 1 --no-kfac --fp32 --sequential > $O/seq_fp32_nokfac.jsonl 2> $O/seq1.err || { echo "seq1 rc=$?"; tail -3 $O/seq1.err; exit 1; }
cat $O/seq_fp32_nokfac.jsonl
timeout -k 10 200 python -u tools/graph_nan_probe.py --steps 6 --image 224 --batch 32 --fused-sgd 1 --no-kfac --sequential > $O/seq_bf16_nokfac.jsonl 2> $O/seq2.err || { echo "seq2 rc=$?"; tail -3 $O/seq2.err; exit 1; }
cat $O/seq_bf16_nokfac.jsonl
timeout -k 10 300 python -u tools/graph_nan_probe.py --steps 14 --image 224 --batch 32 --fused-sgd 1 --factor-steps 4 --fp32 --sequential > $O/seq_fp32_kfac.jsonl 2> $O/seq3.err || { echo "seq3 rc=$?"; tail -3 $O/seq3.err; exit 1; }
cat $O/seq_fp32_kfac.jsonl
