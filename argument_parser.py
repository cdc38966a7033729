#!/usr/bin/env python3
"""Shared CLI of the demos.

The reference's seven flags (``argument_parser.py:6-28`` of
ammunk/distributed-training-pytorch) keep their names, choices and defaults;
everything the reference hard-codes (batch 256, 1000 iterations, lr 1e-3,
1 h timeout, wandb project/group) becomes a flag with the same default, plus
the MI355X engine knobs.
"""
import argparse
import random


def build_parser(description: str | None = None) -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description=description)
    # --- reference flags -----------------------------------------------------
    p.add_argument("--dataloader", choices=["distributed", "standard"], type=str, default="distributed")
    p.add_argument("--backend", choices=["nccl", "mpi", "gloo"], type=str, default="nccl",
                   help="nccl = RCCL on ROCm; gloo for CPU plumbing; mpi needs an MPI-enabled torch")
    p.add_argument("--torchrun", action="store_true", help="Specify we are using torchrun to distribute jobs")
    p.add_argument("--use_node_rank", action="store_true",
                   help="Use NODE_RANK*TASKS_PER_NODE+SLURM_LOCALID as the global rank (per-node srun launches)")
    p.add_argument("--seed", default=random.randint(0, 2 ** 32 - 1), type=int)
    p.add_argument("--num_workers", default=0, type=int)
    p.add_argument("--dry_run", action="store_true", help="Dry run (WANDB_MODE=dryrun)")
    # --- workload (reference constants as defaults) ----------------------------
    p.add_argument("--iters", type=int, default=1000, help="training iterations (demo.py:88)")
    p.add_argument("--batch_size", type=int, default=256, help="per-rank batch (demo.py:145)")
    p.add_argument("--lr", type=float, default=1e-3)
    p.add_argument("--optimizer", choices=["adam", "sgd"], default="adam")
    p.add_argument("--momentum", type=float, default=0.0)
    p.add_argument("--weight_decay", type=float, default=0.0)
    p.add_argument("--loss", choices=["mse", "ce"], default="mse")
    p.add_argument("--n_samples", type=int, default=512, help="ToyData size (toy_model_and_data.py:29)")
    p.add_argument("--per_rank_data", action="store_true",
                   help="each rank draws its own dataset (the reference's unseeded behaviour)")
    p.add_argument("--hidden", type=int, default=10)
    p.add_argument("--depth", type=int, default=3, help="number of hidden Linear(h,h) layers")
    p.add_argument("--precision", choices=["fp32", "bf16"], default="fp32",
                   help="fp32 = the reference (precision=32); bf16 = bf16 matmul operands with fp32 "
                        "accumulation, fp32 master weights and optimizer (fused toy kernels have bf16 "
                        "instances; wide models run bf16 on the MFMA GEMM path)")
    p.add_argument("--timeout_min", type=float, default=60.0, help="process-group timeout (demo.py:27)")
    # --- MI355X engine ---------------------------------------------------------
    p.add_argument("--device", choices=["auto", "cuda", "cpu"], default="auto")
    p.add_argument("--engine", choices=["fused", "module", "stock"], default="fused",
                   help="fused: FusedTrainer (1 kernel/step or persistent); module: nn.Module + FlatDDP + "
                        "fused kernels per op; stock: plain PyTorch eager DDP (the comparison baseline)")
    p.add_argument("--comm", choices=["auto", "rccl", "xgmi", "host"], default="auto")
    p.add_argument("--launch", choices=["persistent", "graph", "eager"], default="persistent")
    # 200: a launch's ~15 us of launch + completion spread over 200 steps (50: 67.5 M samples/s
    # on the fused engine, profiles/r6_native_log/); every step is still logged, one block per launch
    p.add_argument("--steps_per_launch", type=int, default=200,
                   help="iterations per kernel launch / graph (also the host logging granularity)")
    p.add_argument("--sampler", choices=["torch", "device"], default="torch",
                   help="torch: the reference's exact DistributedSampler order (randperm per epoch, read by "
                        "the kernels from a device ring the host fills ahead); device: keyed Feistel shuffle")
    p.add_argument("--log_every", type=int, default=200,
                   help="steps per host read-back of the per-step losses (each step is still logged)")
    p.add_argument("--log_dir", type=str, default=None)
    p.add_argument("--project", type=str, default="distributed tester")
    p.add_argument("--checkpoint_dir", type=str, default=None)
    p.add_argument("--checkpoint_every", type=int, default=0)
    p.add_argument("--resume", action="store_true")
    p.add_argument("--fail_at_iter", type=int, default=None, help="fault injection (first attempt only)")
    p.add_argument("--fail_rank", type=int, default=0)
    p.add_argument("--check_replicas", action="store_true", help="verify DP replicas are bitwise identical")
    p.add_argument("--no_progress", action="store_true")
    return p


def get_args(argv=None):
    return build_parser().parse_args(argv)


if __name__ == "__main__":
    print(get_args())
