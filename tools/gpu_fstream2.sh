set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"; cd "$R"
for fs in 1 0 1 0; do
  KFAC_FACTOR_STREAM=$fs timeout -k 10 300 python3 bench.py --graphs 0 --grad-set-to-none 0 > gpurun_out/fs2_$fs.json 2>/dev/null || exit $?
  tail -1 gpurun_out/fs2_$fs.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('eager fstream=$fs', d['ms_per_step'], d['value'], 'sgd', d['sgd_ms_per_step'])"
done
