#!/bin/bash
# round-3 diagnostics: phase stamps, K=20 wall breakdown (+ kernel trace), demo sampler A/B,
# host profile of the Lightning-style Trainer loop
export TMPDIR=/tmp WANDB_MODE=dryrun
mkdir -p gpurun_out/r3g
bash scripts/gpu_steps.sh \
  "90|r3g/stamps|python scripts/prof_stamps.py" \
  "90|r3g/k20_breakdown|python scripts/k20_breakdown.py 20 30" \
  "150|r3g/k20_rocprof|timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r3g/prof -o k20 -- python3 scripts/k20_breakdown.py 20 30" \
  "120|r3g/demo_torch|python demo.py --iters 1000 --seed 0 --no_progress" \
  "120|r3g/demo_device|python demo.py --iters 1000 --seed 0 --no_progress --sampler device" \
  "180|r3g/lt_prof|python -m cProfile -o gpurun_out/r3g/lt.prof demo_pytorch_lightning.py --gpus 1 --steps 1000 --no_progress --root_dir /tmp/lt" \
  "60|r3g/lt_stats|python -c \"import pstats; pstats.Stats('gpurun_out/r3g/lt.prof').sort_stats('tottime').print_stats(30)\"" \
  "120|r3g/demo_prof|python -m cProfile -o gpurun_out/r3g/demo.prof demo.py --iters 1000 --seed 0 --no_progress" \
  "60|r3g/demo_stats|python -c \"import pstats; pstats.Stats('gpurun_out/r3g/demo.prof').sort_stats('tottime').print_stats(30)\""
