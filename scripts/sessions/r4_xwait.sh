#!/bin/bash
# round 4: overhead of the exchange-wait diagnostic (s_memrealtime per exchange + one
# atomic per launch): share-GPU rehearsals at W = 2 and 8, K = 2000, with and without it
export TMPDIR=/tmp
D=${1:-r4xw2}
mkdir -p gpurun_out/$D
export V=$PWD/distributed_training_pytorch_amd/_lib/var_xwait0/libdtp.so
bash scripts/gpu_steps.sh \
  "900|$D/ab|for r in 1 2 3; do for w in 2 8; do for lib in default \$V; do if [ \$lib = default ]; then unset DTP_LIB; else export DTP_LIB=\$lib; fi; echo \"W=\$w lib=\${lib##*/_lib/}\"; timeout 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node \$w --master-addr 127.0.0.1 --master-port \$((29700 + r * 10 + w)) bench.py --gpus \$w --share-gpu --steps 2000 --warmup 100 | grep -o '\"ms_per_step\": [0-9.e-]*'; done; done; done"
