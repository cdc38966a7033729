#!/bin/bash
# Multi-rank rehearsal of bench.py on a one-GPU box (every rank on cuda:0, gloo host PG,
# in-kernel exchange through IPC-mapped buffers of the same device). Not a scaling number.
# usage: bash scripts/rehearse_share_gpu.sh "2 4 8" [extra bench args]  -> gpurun_out/rehearse_W*.json
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd "$R"
for W in $1; do
  port=$((29500 + W))
  timeout -k 10 240 python -m torch.distributed.run --nnodes 1 --nproc-per-node "$W" --master-addr 127.0.0.1 \
    --master-port "$port" bench.py --gpus "$W" --share-gpu --steps 2000 --warmup 200 ${2} \
    > "gpurun_out/rehearse_W$W.json" 2> "gpurun_out/rehearse_W$W.err" || { echo "W=$W failed"; tail -n 20 "gpurun_out/rehearse_W$W.err"; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/rehearse_W$W.json') if l.startswith('{')][-1]); print($W, round(d['ms_per_step']*1e3,3), round(d['value']/1e6,1), d['config']['comm'])"
done
