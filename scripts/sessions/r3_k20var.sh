#!/bin/bash
# K=20 line variance: kernel time of the timed 20-step launch vs the wall line, 8 fresh processes
export TMPDIR=/tmp
mkdir -p gpurun_out/k20v
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/k20v/p$i -o k20 -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/k20v/bench_$i.log 2>&1 || exit $?
done
# the Lightning demo on the fused engine, with the steady-state rate (first launch of 10 steps excluded)
timeout -k 10 120 python demo_pytorch_lightning.py --gpus 1 --steps 20000 --seed 0 --no_progress --root_dir /tmp/ltf > gpurun_out/k20v/lightning_fused.log 2>&1
