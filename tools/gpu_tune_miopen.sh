# Build the shipped MIOpen find-db: independent MIOpen find runs over the
# bench's convolutions (channels_last for this framework, NCHW for the
# reference harness), merged keeping each solver's best time.
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/tune"; cd "$R"
for layout in cl nchw; do
  extra=""; [ $layout = nchw ] && extra="--no-channels-last"
  for i in 1 2 3 4; do
    d="$R/gpurun_out/tune/${layout}_$i"; mkdir -p $d
    MIOPEN_USER_DB_PATH=$d timeout -k 10 300 python3 bench.py --steps 5 --warmup 3 --cudnn-benchmark 1 --no-kfac $extra > $d/run.json 2> $d/run.err || exit $?
    echo "$layout $i done"
  done
done
python3 tools/merge_miopen_fdb.py gpurun_out/tune/merged.ufdb.txt gpurun_out/tune/*/*.ufdb.txt || exit $?
mkdir -p gpurun_out/tune/db
cp gpurun_out/tune/merged.ufdb.txt gpurun_out/tune/db/$(basename $(ls gpurun_out/tune/cl_1/*.ufdb.txt))
cp gpurun_out/tune/cl_4/*.udb.txt gpurun_out/tune/db/
cat gpurun_out/tune/nchw_4/*.udb.txt >> gpurun_out/tune/db/$(basename $(ls gpurun_out/tune/cl_4/*.udb.txt))
export MIOPEN_USER_DB_PATH=$R/gpurun_out/tune/db
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --steps 40 --warmup 10 --no-kfac > gpurun_out/tune/check_$i.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/tune/check_$i.json').read().strip().splitlines()[-1]); print('check', $i, d['ms_per_step'])"
done
