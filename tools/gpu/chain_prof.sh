set -o pipefail
export TMPDIR=/tmp
out=$PWD/gpurun_out/r6q; mkdir -p $out
for cfg in "4608 1" "4608 3"; do
  set -- $cfg
  raw=/tmp/chain_$1_$2; rm -rf $raw
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $raw -o run -- python3 tools/eigh_probe.py --sizes $1 --count $2 --reps 2 --no-acc > $out/probe_$1_$2.json 2> $out/err_$1_$2.txt || exit $?
  csv=$(find $raw -name '*kernel_trace.csv' | head -n 1)
  python3 tools/chain_trace.py $csv --last-ms 250 > $out/chain_$1_$2.txt || exit $?
done
