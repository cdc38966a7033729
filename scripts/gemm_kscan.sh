#!/bin/bash
# NN bf16: per-tile fixed cost vs K (same 8192x4096 output: 512 tiles = 2 per CU) and vs
# tiles per CU (same K), ours against hipBLASLt (torch.matmul)
D=${1:-gemmk}
mkdir -p gpurun_out/$D
for shape in "8192 4096 2048" "8192 4096 4096" "8192 4096 8192" "8192 4096 16384" "8192 8192 4096" "16384 8192 4096" "8192 8192 8192"; do
  for w in fast torch; do
    timeout -k 10 60 python scripts/gemm_one.py $shape NN 50 $w || exit $?
  done
done
