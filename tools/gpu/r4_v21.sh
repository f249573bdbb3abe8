#!/bin/bash
# Round 4: (1) the driver's bench command (fp32 + SGD + bf16 secondary with
# replay counts), smoke, and a 2-rank gloo rehearsal of the multi-rank bench
# path -- on the suite-verified kernels; (2) GemmConv1x1 with a slab-reduced
# weight gradient (PyTorch-level change, no new kernels): 1x1 conv probe,
# graph interleave test, poison audit in the bench's bf16 mode, bf16 bench.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4z; mkdir -p $O
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --same-device --steps 10 --warmup 3 --secondary-bf16 0 --baseline 0 > $O/rehearsal_gloo_w2.json 2> $O/rehearsal.err || { tail -20 $O/rehearsal.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/rehearsal_gloo_w2.json').read().strip().splitlines()[-1]);print('w2', d['value'], d['kind_ms'], d.get('params_finite'))"
python3 -c "import json;d=json.loads(open('$O/bench_driver_cmd.json').read().strip().splitlines()[-1]);print(d['value'],d['kind_ms'],d.get('kfac_overhead_ms'),d.get('step_graphs'));print(d['bf16'])"
timeout -k 10 200 python3 -u tools/conv1x1_probe.py --bf16 > $O/conv1x1_bf16.jsonl 2> $O/conv.err || exit 1
tail -1 $O/conv1x1_bf16.jsonl
timeout -k 10 200 python3 -u tools/conv1x1_probe.py > $O/conv1x1_fp32.jsonl 2>> $O/conv.err || exit 1
tail -1 $O/conv1x1_fp32.jsonl
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_graphs_refresh_gpu.py tests/test_conv.py > $O/pytest_graphs.log 2>&1 || { tail -20 $O/pytest_graphs.log; exit 1; }
tail -2 $O/pytest_graphs.log
timeout -k 10 400 python3 -u tools/graph_oop_audit.py --bf16 --conv-mode gemm --deterministic 0 > $O/audit_bf16_gemm.jsonl 2> $O/audit.err || exit 1
tail -2 $O/audit_bf16_gemm.jsonl | cut -c1-400
timeout -k 10 400 python3 bench.py --bf16 --steps 100 --warmup 10 --baseline 0 > $O/bench_bf16.json 2> $O/bench_bf16.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_bf16.json'));print('bf16', d['value'], d['kind_ms'], d.get('step_graphs'), d.get('host_issue_ms'), d['params_finite'])"
for m in miopen gemm; do
  timeout -k 10 400 python3 bench.py --steps 100 --warmup 10 --secondary-bf16 0 --conv1x1 $m > $O/bench_fp32_$m.json 2>> $O/bench_fp32.err || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_fp32_$m.json'));print('fp32 $m', d['value'], d['kind_ms'], d.get('sgd_ms_per_step'), d['params_finite'])"
done
du -sh gpurun_out
