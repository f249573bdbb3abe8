# A/B of the factor side stream in the 2-rank gloo rehearsal (ranks share
# the one GPU), same box, alternating order.
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"; cd "$R"
out=gpurun_out/fstream_w2.jsonl; : > $out
port=29531
for fs in 1 0 1 0; do
  KFAC_FACTOR_STREAM=$fs timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 --steps 30 --warmup 5 --backend gloo --same-device --baseline 0 --batch-size 8 --image-size 112 --kfac-inv-update-steps 10 --phase-timing > gpurun_out/fs.json 2> gpurun_out/fs_$fs.err || { tail -30 gpurun_out/fs_$fs.err; exit 1; }
  echo "{\"factor_stream\": $fs, \"r\": $(tail -1 gpurun_out/fs.json)}" >> $out
  python3 -c "import json; d=json.loads(open('gpurun_out/fs.json').read().strip().splitlines()[-1]); print('fs=$fs', d['value'], d['ms_per_step'], d.get('phase_ms_per_step'))"
  port=$((port+1))
done
