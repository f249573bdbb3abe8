# Add NCHW entries to the shipped MIOpen db, then measure the reference and
# this framework under the same harness defaults.
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/ref2/db"; cd "$R"
cp miopen_db/* gpurun_out/ref2/db/
export MIOPEN_USER_DB_PATH=$R/gpurun_out/ref2/db
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 3 --cudnn-benchmark 1 --no-kfac --no-channels-last > gpurun_out/ref2/find_$i.json 2>/dev/null || exit $?
done
export KFAC_REFERENCE_PATH="$R/_refbench"
timeout -k 10 500 python3 bench.py --impl reference --no-channels-last --steps 100 --warmup 10 > gpurun_out/ref2/bench_reference.json 2> gpurun_out/ref2/bench_reference.err || exit $?
tail -1 gpurun_out/ref2/bench_reference.json | cut -c1-300; grep -o '"sgd_ms_per_step[^,]*' gpurun_out/ref2/bench_reference.json
for i in 1 2; do
timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 --phase-timing > gpurun_out/ref2/bench_$i.json 2> gpurun_out/ref2/bench_$i.err || exit $?
tail -1 gpurun_out/ref2/bench_$i.json | cut -c1-260; grep -o '"sgd_ms_per_step[^,]*\|"phase_ms_per_step[^}]*' gpurun_out/ref2/bench_$i.json
done
