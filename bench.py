#!/usr/bin/env python3
"""Headline benchmark: samples/sec (whole node) of the toy-MLP DDP demo.

Workload (BASELINE.md / SURVEY.md §6): two independent ToyModels (X, Y) trained
per iteration -- Linear(2,10), 3x Linear(10,10), Linear(10,1), LeakyReLU --
MSE loss, Adam(lr=1e-3), fp32, per-rank batch 256, DistributedSampler
shuffle, global mean loss reduced every step.  One "step" = one iteration of
``demo.py:99-128`` on every rank: sample the batch, forward+backward both
models, all-reduce gradients, Adam update of both models, reduce the loss.

Scaling: ``strong`` (default) is the reference workload at every N: ONE fixed
512-sample set split by the DistributedSampler, per-rank batch ceil(512/W)
capped at 256 -> 256 / 256 / 128 / 64 at W = 1 / 2 / 4 / 8, global batch 256
(W=1) or 512 (``demo.py:141-148``; BASELINE.md workload table).  ``weak`` keeps
512 samples per rank instead (n = 512*W, per-rank batch 256) -- a config the
reference never ran, kept as an extra.

Usage: python bench.py --gpus N --steps K --warmup W
N > 1 runs under an outer torchrun, or -- without one (no WORLD_SIZE in the
environment) -- bench.py starts its own N ranks (``self_launch``).
Prints ONE JSON line (rank 0's).
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from distributed_training_pytorch_amd.data.sampler import SamplerGeometry  # noqa: E402
from distributed_training_pytorch_amd.data.toy_data import ToyData  # noqa: E402
from distributed_training_pytorch_amd.engine.fused_trainer import EngineConfig, FusedTrainer  # noqa: E402
from distributed_training_pytorch_amd.models.toy import ToyModel  # noqa: E402
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC, MlpSpec  # noqa: E402
from distributed_training_pytorch_amd.ops.optim import OptimConfig  # noqa: E402
from distributed_training_pytorch_amd.parallel import comm_util  # noqa: E402
from distributed_training_pytorch_amd.runtime import bootstrap  # noqa: E402

METRIC = "samples/sec (whole node) toy MLP DDP at 1/2/4/8 MI355X; scaling efficiency"
# The reference publishes no numbers, so the baseline is its loop
# re-enacted on stock PyTorch-ROCm eager (`bench.py --impl stock`), measured on one
# MI355X: 104,998 samples/s (profiles/r1_bench_stock.json).  For N > 1 the
# denominator is that number times N -- stock DDP with PERFECT linear scaling,
# an upper bound on what the stock loop could reach (only 1 GPU is available to
# measure it on).
STOCK_SAMPLES_PER_S_1GPU = 104998.36


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--impl", choices=["native", "stock"], default="native")
    ap.add_argument("--launch", choices=["persistent", "graph", "eager"], default="persistent")
    ap.add_argument("--steps-per-launch", type=int, default=1000)
    ap.add_argument("--comm", choices=["auto", "rccl", "xgmi"], default="auto")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="strong")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--sampler", choices=["torch", "device"], default="torch",
                    help="torch: DistributedSampler's exact order (the reference loader); device: Feistel order")
    ap.add_argument("--precision", choices=["fp32", "bf16"], default="fp32",
                    help="fp32 = the reference's precision=32 (the headline); bf16 = bf16 matmul operands, "
                         "fp32 accumulation / master weights / Adam (BASELINE config 2)")
    ap.add_argument("--cu-mask", choices=["off", "on"], default="off",
                    help="on: run the train kernel on a stream pinned to the first n_models CUs, so its "
                         "code stays in those CUs' instruction cache between launches")
    ap.add_argument("--optimizer", choices=["adam", "sgd"], default="adam",
                    help="adam = the reference's Adam(lr=1e-3); sgd = SGD(lr=1e-2, momentum=0.9) (BASELINE north star)")
    ap.add_argument("--loss", choices=["mse", "ce"], default="mse",
                    help="mse = the reference's MSELoss (2-10-10-10-10-1); ce = cross-entropy over 4 classes "
                         "(2-10-10-10-10-4 head, targets bucketed into 4 classes; BASELINE north star)")
    ap.add_argument("--groups", choices=["auto", "on", "off"], default="auto",
                    help="split-batch step (csrc/grp_core.h): a rank's batch over batch/64 workgroups per model; "
                         "auto = the measured policy")
    ap.add_argument("--stream", choices=["default", "pool"], default="pool",
                    help="pool (default): the run's launches go to a torch pool stream (non-blocking: no implicit "
                         "synchronisation with the legacy default stream); default: the device's default stream. "
                         "Driver-style K=20, 14 fresh processes each, interleaved: median 4.52 vs 4.62 us/step, and "
                         "no 8-10 us outliers (3 of 14 on the default stream; profiles/r6_misc/)")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal only: every rank on cuda:(local_rank %% device_count), gloo process group "
                         "(exercises the multi-rank path on a 1-GPU box; numbers are not scaling numbers)")
    return ap.parse_args()


def cpu_idle_ticks(cpus, window_s: float = 0.03) -> dict:
    """Idle + iowait ticks of each CPU in ``cpus`` over ``window_s`` (/proc/stat); {} when
    unreadable."""
    def snap():
        out = {}
        with open("/proc/stat") as f:
            for line in f:
                if line.startswith("cpu") and line[3:4].isdigit():
                    v = line.split()
                    out[int(v[0][3:])] = int(v[4]) + int(v[5])
        return out

    try:
        a = snap()
        time.sleep(window_s)
        b = snap()
    except (OSError, ValueError, IndexError):
        return {}
    return {c: b[c] - a[c] for c in cpus if c in a and c in b}


def pin_host_thread(dev) -> int | None:
    """Keep this (launching, synchronizing) thread on a CPU of the GPU's NUMA node: the
    K-step call is a launch, a wait and a synchronize, so a remote-node wakeup lands
    inside the timed region.  The CPU comes from the GPU's PCI ``local_cpulist`` within
    this process's allowed set (one local process: idlest first over 30 ms of
    /proc/stat); each local rank takes its own (DTP_BENCH_PIN=set: a group of 4; first:
    the first CPU; 0: no pinning; A/Bs in profiles/r4_gpu/k20_pin_ab.jsonl.log and
    profiles/r4_pin/).  Returns the first CPU of the set, None when the box does not
    expose it."""
    if dev.type != "cuda" or not hasattr(os, "sched_setaffinity"):
        return None
    mode = os.environ.get("DTP_BENCH_PIN", "one")
    try:
        pr = torch.cuda.get_device_properties(dev)
        bdf = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
        spec = open(f"/sys/bus/pci/devices/{bdf}/local_cpulist").read().strip()
        local = set()
        for part in spec.split(","):
            lo, _, hi = part.partition("-")
            local.update(range(int(lo), int(hi or lo) + 1))
        allowed = sorted(local & os.sched_getaffinity(0)) or sorted(os.sched_getaffinity(0))
        # idlest first -- for a single local process only: ranks sampling /proc/stat at
        # different moments would sort differently and could pick the same CPU
        single = int(os.environ.get("LOCAL_WORLD_SIZE", "1")) == 1
        idle = cpu_idle_ticks(allowed) if mode != "first" and single else {}
        if idle:
            allowed = sorted(allowed, key=lambda c: -idle.get(c, 0))  # stable: ties keep CPU order
        g = min(4, len(allowed)) if mode == "set" else 1
        r = int(os.environ.get("LOCAL_RANK", "0"))
        cpus = [allowed[(r * g + k) % len(allowed)] for k in range(g)]
        os.sched_setaffinity(0, set(cpus))
        return cpus[0]
    except (OSError, ValueError, AttributeError, IndexError):
        return None


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(a, argv: list[str]) -> int:
    """``--gpus N > 1`` without a launcher around us: start the N ranks ourselves, the way
    the reference's launch layer does (``torchrun --standalone --nproc_per_node G``,
    /root/reference/hpc_files/virtual_env_hpc_files/distributed_scripts/torchrun_launcher.sh:9-20).

    Runs BEFORE this process touches the GPU (counting devices does not) and never execs:
    the ranks are children of a ``torch.distributed.run`` child on 127.0.0.1.  Their
    stderr passes through; their stdout is read here and rank 0's one JSON line is
    forwarded (anything else the ranks print goes to stderr).  Returns the launcher's
    exit code (non-zero as soon as any rank failed -- torchrun tears the others down)."""
    import subprocess

    ndev = torch.cuda.device_count()
    if ndev and a.gpus > ndev and not a.share_gpu:
        raise SystemExit(f"--gpus {a.gpus} but only {ndev} GPUs are visible (--share-gpu rehearses on fewer)")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    env["DTP_BENCH_CHILD"] = "1"  # a rank never launches again, whatever its env says
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env, text=True)
    json_lines = []
    for line in p.stdout:
        s = line.strip()
        if s.startswith("{") and '"metric"' in s:
            json_lines.append(s)
        else:
            sys.stderr.write(line)
    rc = p.wait()
    if rc == 0 and len(json_lines) != 1:
        sys.stderr.write(f"[bench] expected one JSON line from rank 0, got {len(json_lines)}\n")
        rc = 1
    if json_lines:
        print(json_lines[-1], flush=True)
    return rc


def main():
    a = parse()
    # the collective environment goes in FIRST: HSA reads HSA_ENABLE_IPC_MODE_LEGACY once,
    # at the process's first GPU touch (set_wait_mode below is one), and the self-launched
    # ranks inherit it from this process's environment.  Set later, the IPC mapping of the
    # in-kernel exchange fails and the run measures the RCCL fallback instead.
    ipc_env_at_start = os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")
    bootstrap.configure_collective_env()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ and os.environ.get("DTP_BENCH_CHILD") != "1":
        sys.exit(self_launch(a, sys.argv[1:]))
    if torch.cuda.device_count() > 0:  # counting devices does not initialise the GPU
        from distributed_training_pytorch_amd import _native

        # host threads spin on GPU completion (DTP_WAIT_MODE overrides; before the first
        # GPU touch): the timed region ends in a synchronize, and a spinning waiter
        # returns sooner than an interrupt-woken one (K=20 A/B, 8 interleaved runs
        # each: median 5.55 vs 5.65 us/step, profiles/r2_s3/ab_wait.txt)
        _native.set_wait_mode(os.environ.get("DTP_WAIT_MODE", "spin"))
    # the demos' launch path (runtime/bootstrap.py): torchrun / SLURM / MPI env
    # discovery, device binding, process-group init
    env = bootstrap.detect()
    ndev = torch.cuda.device_count()
    if a.share_gpu and ndev > 0:
        env.local_rank %= ndev
    rank, world = env.rank, env.world_size
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}: launch N>1 with torchrun, or without WORLD_SIZE")
    if os.environ.get("DTP_BENCH_FAIL_RANK", "") == str(rank):  # test hook: one rank dies
        raise SystemExit(f"rank {rank}: forced failure (DTP_BENCH_FAIL_RANK)")
    dev = bootstrap.bind_device(env)
    pinned = pin_host_thread(dev) if os.environ.get("DTP_BENCH_PIN", "one") != "0" else None
    if world > 1 or a.impl == "stock":  # the stock loop wraps its models in torch DDP even at W=1
        bootstrap.init_process_group(env, "gloo" if (a.share_gpu or dev.type == "cpu") else "nccl", dev)
    n = 512 * world if a.scaling == "weak" else 512
    if a.impl == "stock" and (a.loss != "mse" or a.optimizer != "adam"):
        raise SystemExit("--impl stock re-enacts the reference loop: MSE + Adam only")
    ds = ToyData(n=n, seed=a.seed, classes=4 if a.loss == "ce" else 0)
    spec = MlpSpec(2, 10, 5, 4) if a.loss == "ce" else TOY_SPEC
    ocfg = OptimConfig(lr=1e-3) if a.optimizer == "adam" else OptimConfig("sgd", 1e-2, momentum=0.9)

    if a.impl == "stock":
        from distributed_training_pytorch_amd.baselines.stock import StockLoop

        runner = StockLoop(ds, dev, batch=a.batch, seed=a.seed)
        per_rank_batch = min(a.batch, -(-n // world))
        train = runner.train
        sync = (lambda: torch.cuda.synchronize(dev)) if dev.type == "cuda" else (lambda: None)
        cfg_desc = {"launch": "eager", "comm": "rccl DDP + gloo loss reduce" if world > 1 else "none"}
    else:
        if a.cu_mask == "on" and dev.type == "cuda":
            from distributed_training_pytorch_amd import _native

            torch.cuda.set_stream(_native.cu_masked_stream(dev, [0, 1]))
        elif a.stream == "pool" and dev.type == "cuda" and world == 1:
            # one rank only: ranks that share a GPU (--share-gpu) co-schedule their in-kernel
            # exchange across processes, and a second queue per process oversubscribes the
            # hardware queues (the W = 8 rehearsal failed once with it); with several GPUs
            # the default stream is what every multi-rank run so far used
            torch.cuda.set_stream(torch.cuda.Stream(device=dev))
        X, Y = ds.device_tensors(dev)
        geom = SamplerGeometry(n=n, world=world, rank=rank, batch=a.batch, seed=a.seed)
        torch.manual_seed(a.seed)
        if a.loss == "ce":  # the 4-class head: torch.nn.Linear's default init of the same layer shapes
            init = [torch.cat([t.reshape(-1) for lay in [torch.nn.Linear(i, o) for i, o in spec.dims()]
                               for t in (lay.weight.detach(), lay.bias.detach())]) for _ in range(2)]
        else:
            init = [ToyModel().flat_params.detach().clone() for _ in range(2)]
        ecfg = EngineConfig(comm=a.comm, launch=a.launch, steps_per_launch=a.steps_per_launch,
                            precision=a.precision, sampler=a.sampler, groups=a.groups, loss=a.loss)
        runner = FusedTrainer(spec, 2, X, Y, geom, ocfg, ecfg, init_params=init)
        per_rank_batch = geom.batch_size_at(0)
        train = runner.train
        # the xGMI timeout word is checked right after the timed region (check_comm below)
        sync = (lambda: torch.cuda.synchronize(dev)) if dev.type == "cuda" else (lambda: None)
        cfg_desc = {"launch": a.launch, "steps_per_launch": a.steps_per_launch, "comm": runner.comm,
                    "host_cpu": pinned,
                    "sampler": "DistributedSampler order (randperm per epoch)" if a.sampler == "torch"
                    else "Feistel shuffle", "cu_mask": a.cu_mask,
                    "stream": "cu_masked" if a.cu_mask == "on" else (a.stream if world == 1 else "default"),
                    # lanes per sample of the fused step (1, or 2 / 4: csrc/mlp_lanes.h for batches <= 128 / 64)
                    "lanes_per_sample": runner.lanes, "waves_per_cu": runner.kernel_waves,
                    # > 1: the split-batch step (csrc/grp_core.h), CUs per model
                    "workgroups_per_model": runner.groups}

    # the timed region is bracketed by an all-rank barrier + synchronize on both sides;
    # ranks of the in-kernel xGMI engine use the framework's device barrier (one xGMI
    # hop, parallel/xgmi.py:DeviceBarrier) instead of an RCCL collective
    dbar = None
    if world > 1 and a.impl == "native" and getattr(runner, "comm", "") == "xgmi":
        from distributed_training_pytorch_amd.parallel.xgmi import DeviceBarrier

        dbar = DeviceBarrier(dev)

    def sync_barrier():
        """synchronize + all-rank barrier.  The device barrier is queued on the stream
        right behind the work before it, so one synchronize covers both (no extra
        launch-and-wait round trip); a process-group barrier follows the synchronize."""
        if dbar is not None:
            dbar()
            sync()
        else:
            sync()
            comm_util.barrier()

    # warmup (untimed): the W steps, spread over up to 16 launches.  The first few
    # launches of a process pay extra runtime latency; with W = 5 in ONE launch the
    # timed call was only the process's second launch (K = 20, 8 fresh processes each,
    # interleaved: 5.96 vs 5.52 us/step median, profiles/r3_gpu/k20_warmup_launches.jsonl).
    # DTP_BENCH_WARMUP_LAUNCHES overrides the count.
    split = max(1, min(a.warmup, int(os.environ.get("DTP_BENCH_WARMUP_LAUNCHES", "16"))))
    done = 0
    for i in range(split):
        k = (a.warmup - done) // (split - i)
        train(k)
        done += k
    xstats = a.impl == "native" and world > 1 and runner.comm == "xgmi"
    if xstats:
        runner.exchange_stats_reset()  # stream-ordered, covered by the synchronize below
    # no cyclic-GC pass inside the timed region.  (A gc.collect() right before it cost the
    # first timed call ~40 us: the collection walks the whole heap and leaves the launch
    # path's host caches cold; K=20 7.3-10.7 vs 5.3 us/step, profiles/r4_pin/k20_gc_ab.log.)
    gc.disable()
    sync_barrier()
    sync()
    t0 = time.perf_counter()
    train(a.steps)
    sync_barrier()
    t1 = time.perf_counter()
    extra = []
    for _ in range(int(os.environ.get("DTP_BENCH_EXTRA", "0"))):  # diagnostic: more timed calls, same recipe
        sync_barrier()
        sync()
        u0 = time.perf_counter()
        train(a.steps)
        sync_barrier()
        extra.append(round(1e3 * (time.perf_counter() - u0) / a.steps, 5))
    gc.enable()
    if a.impl == "native":  # the instance the run actually launched (the engine exists now)
        cfg_desc.update(lanes_per_sample=runner.lanes, waves_per_cu=runner.kernel_waves,
                        workgroups_per_model=runner.groups)
        if runner.groups_refused:
            cfg_desc["groups_refused"] = runner.groups_refused
    elapsed = comm_util.all_reduce_scalar(t1 - t0, dist.ReduceOp.MAX)
    ms_per_step = 1e3 * elapsed / a.steps
    total_samples = comm_util.all_reduce_scalar(float(per_rank_batch * a.steps))
    value = total_samples / elapsed
    diag = {"extra_ms_per_step": extra} if extra else {}
    if world > 1 and a.impl == "native":
        if runner.comm != "xgmi" and rank == 0:
            sys.stderr.write(f"[bench] W={world}: in-kernel xGMI exchange NOT used (comm={runner.comm}): "
                             f"{runner.comm_fallback_reason}\n")
        # where a multi-GPU step goes (readable from the JSON line alone): the in-kernel
        # exchange's wait (publish -> last peer granule, per rank) and the rest of the step
        diag["comm_fallback_reason"] = runner.comm_fallback_reason
        if xstats:
            st = runner.exchange_stats_full()
            n_ex = max(1, st["exchanges"])
            waits = comm_util.all_gather_scalar(st["wait_us"] / n_ex)
            pubs = comm_util.all_gather_scalar(st["publish_us"] / n_ex)
            diag["exchange_wait_us_per_step"] = max(waits)
            diag["exchange_wait_us_per_step_by_rank"] = [round(v, 3) for v in waits]
            # the step three ways: publishing the granules (first -> last store issued),
            # waiting for the peers' granules, and the rest of the step
            diag["publish_us_per_step"] = max(pubs)
            diag["step_rest_us_per_step"] = 1e3 * ms_per_step - max(waits) - max(pubs)
            diag["compute_us_per_step"] = 1e3 * ms_per_step - max(waits)

    final_loss = None
    if dbar is not None:
        dbar.check()  # raises if a barrier exchange timed out
    if a.impl == "native":
        runner.check_comm()  # raises if any in-kernel exchange of the run timed out
        final_loss = runner.losses(runner.t - 1, runner.t)[0].tolist()
        runner.close()  # process-group barrier before the xGMI buffers are unmapped
        if dbar is not None:
            dbar.close()
    else:
        final_loss = list(runner.last)
        runner.close()

    base = STOCK_SAMPLES_PER_S_1GPU * world
    if rank == 0:
        rec = {
            "metric": METRIC,
            "value": value,
            "unit": "samples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": a.scaling,
            "vs_baseline": (value / base) if (base and a.impl == "native") else None,
            "dtype": a.precision if a.impl == "native" else "fp32",
            "data": "synthetic (ToyData distribution, seeded; random-init ToyModel weights)",
            "config": {
                "model": ("2x ToyModel MLP 2-10-10-10-10-1 LeakyReLU (X,Y), MSE, Adam lr=1e-3"
                          if (a.loss, a.optimizer) == ("mse", "adam") else
                          f"2x ToyModel-shaped MLP 2-10-10-10-10-{spec.out_features} LeakyReLU (X,Y), "
                          f"{'cross-entropy (4 classes)' if a.loss == 'ce' else 'MSE'}, "
                          f"{'Adam lr=1e-3' if a.optimizer == 'adam' else 'SGD lr=1e-2 momentum=0.9'}"),
                "global_batch": per_rank_batch * world,
                "per_rank_batch": per_rank_batch,
                "seq_len": None,
                "parallelism": f"dp{world}",
                "impl": a.impl,
                "dataset_samples": n,
                # the IPC-mode variable as this rank's process found it at start (self-launched
                # ranks inherit it from the parent, which sets it before the launch)
                "ipc_env_at_start": ipc_env_at_start,
                **cfg_desc,
            },
            "final_loss": final_loss,
            **diag,
        }
        print(json.dumps(rec), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
