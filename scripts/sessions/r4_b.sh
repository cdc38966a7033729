#!/bin/bash
# round 4, session b: strong-scaling lanes pick, trainer spec check, split stream diagnosis, bench lines
export TMPDIR=/tmp
D=${1:-r4b}
mkdir -p gpurun_out/$D
bash scripts/gpu_steps.sh \
  "400|$D/tests|python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_lanes_gpu.py tests/test_trainer_fused_gpu.py tests/test_bench_gpu.py" \
  "200|$D/bench_w8|for f in 1 2x8 4x8; do DTP_LANES=\$f python bench.py --scaling weak --batch 256; done; for f in 2 4 4x8; do DTP_LANES=\$f python bench.py --scaling weak --batch 128; done" \
  "300|$D/split|python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_split_fused_gpu.py -k 'not per_stage' && for v in 0 1 0 1; do DTP_SPLIT_LOCAL_LINKS=\$v python -m pytest -q -s tests/test_split_fused_gpu.py -k step_time | grep us/step; done" \
  "200|$D/diag_streams|for m in per_device cumask torch prio; do python scripts/diag_split_streams.py \$m; done" \
  "200|$D/rocprof_cumask|timeout -k 10 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$D/prof_cumask -o cumask -- python3 scripts/diag_split_streams.py cumask" \
  "300|$D/bench_k20|for i in 1 2 3 4 5 6; do DTP_BENCH_PIN=1 python bench.py --steps 20 --warmup 5; DTP_BENCH_PIN=0 python bench.py --steps 20 --warmup 5; done" \
  "100|$D/bench_default|python bench.py" \
  "400|$D/share|for w in 2 4 8; do timeout 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node \$w --master-addr 127.0.0.1 --master-port 2961\$w bench.py --gpus \$w --share-gpu --steps 2000 --warmup 100 || exit 3; done"
