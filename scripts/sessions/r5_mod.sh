#!/bin/bash
# round 5: Trainer module path with the fused (X, Y) batch gather and a cached backward seed:
# the Trainer / loss GPU tests, steady samples/s and a kernel trace
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5mod
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_loss_op.py tests/test_trainer_fused_gpu.py tests/test_entrypoints_gpu.py tests/test_graph_xgmi_gpu.py tests/test_kernels_gpu.py > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python3 demo_pytorch_lightning.py --gpus 1 --steps 3000 --seed 0 --root_dir /tmp/ltm --engine module --no_progress > $O/lt_module.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o lt -- python3 demo_pytorch_lightning.py --gpus 1 --steps 3000 --seed 0 --root_dir /tmp/ltq --engine module --no_progress > $O/lt_rocprof.log 2>&1
