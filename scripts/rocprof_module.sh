# rocprofv3 kernel stats of the module engine and the Lightning-style Trainer (GPU box)
R="${GRAFT_REPO_ROOT:-$(pwd)}"
cd /tmp && export TMPDIR=/tmp WANDB_MODE=dryrun
out="$R/gpurun_out/rocprof_module"
mkdir -p "$out"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/module" -o module -- \
  python3 "$R/demo.py" --engine module --iters 300 --seed 0 --no_progress > "$out/module.log" 2>&1 &&
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/lightning" -o lightning -- \
  python3 "$R/demo_pytorch_lightning.py" --gpus 1 --steps 300 --seed 0 --no_progress --root_dir /tmp/lt > "$out/lightning.log" 2>&1
