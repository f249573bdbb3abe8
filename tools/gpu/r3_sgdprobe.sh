#!/bin/bash
# Round 3: plain PyTorch ResNet-50 forward+backward graph replay vs eager (no K-FAC)
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R"; O=gpurun_out/r3l; mkdir -p $O
run() { name=$1; shift; timeout -k 10 120 python -u tools/graph_sgd_probe.py "$@" > $O/$name.json 2> $O/$name.err; rc=$?; python3 -c "
import json; d=json.loads(open('$O/$name.json').read())
print('$name', 'eager-repeat %.1e'%d['eager_repeat_maxrel'], [(r['replay'], '%.1e'%r['maxrel'], r['n_bad'], r['worst'][0][1]) for r in d['replays']])
" || { echo "$name rc=$rc"; grep -v '^frame' $O/$name.err | grep -i error | head -3; }; [ $rc -eq 0 ] || exit 1; }
for i in 1 2 3; do run cl_det$i; done
for i in 1 2; do run cl_nodet$i --nodet; done
for i in 1 2 3; do run nchw$i --nchw; done
for i in 1 2; do run sidewarm$i --side-warmup 2; done
for i in 1 2; do run nocudnn$i --no-cudnn; done
