# Re-entry check after a container restore: full -m gpu suite, smoke, bench,
# then the eigensolver lane probe under several hardware-queue counts.
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"; cd "$R"
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --phase-timing > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
tail -1 gpurun_out/bench.json
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q PROBE_CONFIGS="1:8:100000,1:4:4608,1:8:4608,1:12:4608,1:8:2304" \
    timeout -k 10 300 python3 -u tools/eigh_lanes_probe.py > gpurun_out/eigh_lanes_q$q.jsonl 2> gpurun_out/eigh_lanes_q$q.err || exit $?
done
