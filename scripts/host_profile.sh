# cProfile of the host side of the module engine and the Lightning-style Trainer (GPU box)
mkdir -p gpurun_out
export WANDB_MODE=dryrun
timeout -k 10 120 python -m cProfile -s tottime demo.py --engine module --iters 500 --seed 0 --no_progress > gpurun_out/prof_module.txt 2>&1 &&
timeout -k 10 120 python -m cProfile -s tottime demo_pytorch_lightning.py --gpus 1 --steps 500 --seed 0 --no_progress --root_dir /tmp/lt > gpurun_out/prof_lightning.txt 2>&1 &&
DTP_TRACE=1 timeout -k 10 120 python demo.py --engine module --iters 500 --seed 0 --no_progress > gpurun_out/trace_module.txt 2>&1
