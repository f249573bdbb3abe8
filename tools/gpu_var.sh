# Run-to-run variance of the bench on one box (fresh MIOpen state first).
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/var"; cd "$R"
for i in 1 2 3; do
  for z in 1 0; do
    timeout -k 10 300 python3 bench.py --steps 60 --warmup 10 --grad-set-to-none $z > gpurun_out/var/b_${i}_${z}.json 2> gpurun_out/var/b_${i}_${z}.err || exit $?
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/var/b_${i}_${z}.json').read().strip().splitlines()[-1]); print($i, $z, d['value'], d['ms_per_step'], d.get('sgd_ms_per_step'))"
  done
done
ls ~/.config/miopen ~/.cache/miopen 2>/dev/null | head
