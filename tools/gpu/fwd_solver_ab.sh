# Which MIOpen bf16 forward solver makes layer4.0.conv2 (512 -> 512, 3x3,
# stride 2, 14x14) nondeterministic: the bf16 twin probe (--fwd-check) with
# the tuned find-db entry cut to one solver at a time.
set -o pipefail
out=gpurun_out/fwdsolver; mkdir -p $out
key='512-14-14-3x3-512-7-7-32-1x1-2x2-1x1-0-NHWC-NHWC-NHWC-BF16-F'
for keep in ConvHipImplicitGemmGroupFwdXdlops ConvAsmImplicitGemmGTCDynamicFwdXdlopsNHWC; do
  db=/tmp/db_$keep; rm -rf $db; cp -r miopen_db $db
  python3 - "$db" "$key" "$keep" <<'PY'
import glob, sys
db, key, keep = sys.argv[1:]
f = glob.glob(db + '/*.ufdb.txt')[0]
lines = open(f).read().splitlines()
for i, l in enumerate(lines):
    if l.startswith(key + '='):
        items = [it for it in l.split('=', 1)[1].split(';') if it.startswith(keep + ':')]
        lines[i] = key + '=' + ';'.join(items)
open(f, 'w').write('\n'.join(lines) + '\n')
PY
  MIOPEN_USER_DB_PATH=$db KFAC_CONV_DETERMINISTIC_BF16=1 timeout -k 10 200 python -u tools/determinism_probe.py --cudnn-det 0 --steps 2 --fwd-check > $out/$keep.log 2>&1 || exit $?
  echo "$keep: $(grep -o '"first_fwd_mismatch": [^}]*' $out/$keep.log)"
done
