#!/bin/bash
# round 4: Adam with hardware sqrt / reciprocal + one correction step (DTP_ADAM_FAST) vs the
# precise-division build -- interleaved steady-state A/B, and the variant's numerics
export TMPDIR=/tmp
D=${1:-r4adam}
mkdir -p gpurun_out/$D
V=distributed_training_pytorch_amd/_lib/var_adamfast/libdtp.so
bash scripts/gpu_steps.sh \
  "300|$D/ab|for r in 1 2 3; do for lib in default \$PWD/$V; do for b in 256 64; do if [ \$lib = default ]; then unset DTP_LIB; else export DTP_LIB=\$lib; fi; echo \"lib=\$lib batch=\$b\"; python bench.py --scaling weak --batch \$b --steps 2000 --warmup 100; done; done; done" \
  "300|$D/k20|for r in 1 2 3 4; do for lib in default \$PWD/$V; do if [ \$lib = default ]; then unset DTP_LIB; else export DTP_LIB=\$lib; fi; echo \"lib=\$lib\"; python bench.py --steps 20 --warmup 5; done; done" \
  "400|$D/tests|DTP_LIB=\$PWD/$V python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lanes_gpu.py tests/test_kernels_gpu.py"
