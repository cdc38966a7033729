"""MI355X-native distributed-training harness (gfx950 / CDNA4, PyTorch-ROCm + HIP + RCCL/xGMI).

Capabilities of ammunk/distributed-training-pytorch, re-designed MI355X-first:
fused HIP train-step kernels, device-side sampling, hipGraph / persistent
multi-step execution, flat-buffer data parallelism over RCCL or an in-kernel
xGMI one-shot all-reduce, layer-split model parallelism with peer hand-off,
a Lightning-style Trainer, launch/bootstrap for torchrun / SLURM / MPI / PBS.
"""
__version__ = "0.1.0"

from .ops.mlp import MlpSpec, TOY_SPEC  # noqa: F401
