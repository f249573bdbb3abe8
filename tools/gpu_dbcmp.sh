set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/dbcmp"; cd "$R"
for i in 1 2 3; do
  for v in ship merged none; do
    case $v in ship) db=$R/miopen_db;; merged) db=$R/tools/_mdb_merged;; none) db=$R/gpurun_out/dbcmp/empty_$i; mkdir -p $db;; esac
    MIOPEN_USER_DB_PATH=$db timeout -k 10 300 python3 bench.py --steps 40 --warmup 10 --no-kfac > gpurun_out/dbcmp/${v}_$i.json 2>/dev/null || exit $?
    python3 -c "import json; d=json.loads(open('gpurun_out/dbcmp/${v}_$i.json').read().strip().splitlines()[-1]); print('$v', $i, d['ms_per_step'])"
  done
done
