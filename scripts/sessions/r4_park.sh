#!/bin/bash
# round 4: column-major conflict-free dW tile park (ds_write_b128) vs the row-major
# ds_write_b32 park -- numerics suites, then interleaved K=2000 A/B at batch 256 / 64
export TMPDIR=/tmp
D=${1:-r4park}
mkdir -p gpurun_out/$D
export V=$PWD/distributed_training_pytorch_amd/_lib/var_oldpark/libdtp.so
bash scripts/gpu_steps.sh \
  "500|$D/tests|python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_lanes_gpu.py tests/test_split_fused_gpu.py tests/test_bf16_gpu.py tests/test_bench_gpu.py tests/test_xgmi_gpu.py" \
  "300|$D/ab|for r in 1 2 3; do for lib in default \$V; do for b in 256 64; do if [ \$lib = default ]; then unset DTP_LIB; else export DTP_LIB=\$lib; fi; echo \"lib=\${lib##*/_lib/} batch=\$b\"; python bench.py --scaling weak --batch \$b --steps 2000 --warmup 100 | grep -o '\"ms_per_step\": [0-9.e-]*'; done; done; done"
