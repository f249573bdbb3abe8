# Build a MIOpen find-db for the bench config and check that immediate mode
# (cudnn.benchmark=False) with that db gives stable step times.
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/mdb/db"; cd "$R"
export MIOPEN_USER_DB_PATH="$R/gpurun_out/mdb/db"
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --steps 40 --warmup 10 --grad-set-to-none 1 --cudnn-benchmark 1 --no-kfac > gpurun_out/mdb/find_$i.json 2> gpurun_out/mdb/find_$i.err || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/mdb/find_$i.json').read().strip().splitlines()[-1]); print('find', $i, d['ms_per_step'])"
done
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --steps 40 --warmup 10 --grad-set-to-none 1 --cudnn-benchmark 0 --no-kfac > gpurun_out/mdb/imm_$i.json 2> gpurun_out/mdb/imm_$i.err || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/mdb/imm_$i.json').read().strip().splitlines()[-1]); print('immediate+db', $i, d['ms_per_step'])"
done
unset MIOPEN_USER_DB_PATH
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 40 --warmup 10 --grad-set-to-none 1 --cudnn-benchmark 0 --no-kfac > gpurun_out/mdb/nodb_$i.json 2> gpurun_out/mdb/nodb_$i.err || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/mdb/nodb_$i.json').read().strip().splitlines()[-1]); print('immediate no db', $i, d['ms_per_step'])"
done
ls -la gpurun_out/mdb/db
