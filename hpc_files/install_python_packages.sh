#!/bin/bash
# Create ./virtual_env for the harness (run as a SLURM job by job_submitter.sh).
# PyTorch must be a ROCm build (the MI355X image ships torch 2.10+rocm7.0); the
# venv inherits it with --system-site-packages so no GPU wheel has to be fetched.
set -e
python -m venv --system-site-packages virtual_env
source virtual_env/bin/activate
if [[ -f requirements.txt ]]; then
  pip install --no-deps -r requirements.txt || echo "offline: using the system site-packages"
fi
python -c "import torch; print('torch', torch.__version__, 'hip', torch.version.hip)"
# build the HIP kernels for gfx950 in-tree
python -m distributed_training_pytorch_amd.build
