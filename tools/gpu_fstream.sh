set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"; cd "$R"
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for g in 1 0; do
for fs in 1 0 1 0; do
  KFAC_FACTOR_STREAM=$fs timeout -k 10 300 python3 bench.py --graphs $g --phase-timing > gpurun_out/fs_${g}_$fs.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/fs_${g}_$fs.json').read().strip().splitlines()[-1]); print('graphs=$g fstream=$fs', d['ms_per_step'], d['value'], d['sgd_ms_per_step'], {k: round(v,3) for k,v in d['phase_ms_per_step'].items()})"
done
done
