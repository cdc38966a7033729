set -o pipefail
mkdir -p gpurun_out
export WANDB_MODE=dryrun
run() { name=$1; shift; echo "== $name"; timeout -k 10 120 python "$@" --no_progress > gpurun_out/ep_$name.log 2>&1 || { echo "FAIL $name"; tail -5 gpurun_out/ep_$name.log; return 1; }; grep "summary" gpurun_out/ep_$name.log | tail -1; }
run fused demo.py --iters 1000 --seed 0 &&
run module demo.py --engine module --iters 1000 --seed 0 &&
run stock demo.py --engine stock --iters 1000 --seed 0 &&
run split_mb1 demo_one_model_multi_gpu.py --allow_shared_gpu --iters 1000 --seed 0 &&
run split_mb4 demo_one_model_multi_gpu.py --allow_shared_gpu --microbatches 4 --iters 1000 --seed 0 &&
run lightning demo_pytorch_lightning.py --gpus 1 --steps 1000 --seed 0 --root_dir /tmp/lt
