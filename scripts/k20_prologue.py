"""Where the fixed cost of one 20-step launch of the split-batch step goes (the driver's
K = 20 line): the PROF instance's launch-level stamps (mlp_train.hip lanes kernel, row 0
slots 20 / 18 / 19 / 22 / 23 / 29 / 24 / 21) and its per-step phase stamps (rows 0..7).

Prints, per launch, cycles (s_memtime, shader clock) of: the prologue (entry -> global
loads consumed -> weight scatter -> Adam table -> loop start), step 0 against the mean of
steps 1..6, the exchange inside step 0 against steady steps, the mean of steps 7..19 and the
write-back.  Launch 0 is the process's first launch of the instance (cold instruction cache);
the others follow 16 warm-up launches like bench.py's.  GPU only; one JSON line per launch."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_pytorch_amd import _native as nat  # noqa: E402
from distributed_training_pytorch_amd.data.sampler import SamplerGeometry  # noqa: E402
from distributed_training_pytorch_amd.data.toy_data import ToyData  # noqa: E402
from distributed_training_pytorch_amd.engine.fused_trainer import FusedTrainer  # noqa: E402
from distributed_training_pytorch_amd.models.toy import ToyModel  # noqa: E402
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC  # noqa: E402


def one(tr, lib, n, label):
    nblk = 8 * tr.groups
    prof = torch.zeros(nblk * 8 * 32, dtype=torch.int64, device=tr.device)
    nat.check(lib.dtp_train_engine_profile(tr._engine_handle(), n, tr.t, nat.ptr(prof), nat.stream_ptr()),
              "engine profile")
    torch.cuda.synchronize()
    tr.t += n
    st = prof.view(nblk, 8, 32).cpu().tolist()
    r0 = st[0][0]
    steps = [st[0][k][0] for k in range(8)]
    ex = [st[0][k][5] - st[0][k][4] for k in range(8)]
    members_end = [st[8 * k][0][24] for k in range(tr.groups)]
    rec = {
        "launch": label,
        "prologue_issue": r0[18] - r0[20],      # entry -> every prologue load issued (incl. the status wait)
        "prologue_loads": r0[19] - r0[20],      # entry -> first barrier (params, moments, dataset in LDS)
        "prologue_scatter": r0[22] - r0[19],    # weight scatter into the blocks
        "prologue_adam_tab": r0[23] - r0[22],   # the Adam table rows into LDS
        "prologue_to_loop": r0[29] - r0[23],    # lane bases, the last barrier
        "prologue_total": r0[29] - r0[20],
        "step0": steps[1] - steps[0],
        "steps1_6_mean": (steps[7] - steps[1]) / 6,
        "exchange_step0": ex[0],
        "exchange_steps1_6_mean": sum(ex[1:7]) / 6,
        "steps7_end_mean": (r0[24] - steps[7]) / (n - 7),
        "writeback": r0[21] - r0[24],
        "kernel_entry_to_exit": r0[21] - r0[20],
        "member_end_skew": max(members_end) - min(members_end),
    }
    print(json.dumps(rec), flush=True)


def main():
    dev = torch.device("cuda", 0)
    X, Y = ToyData(n=512, seed=0).device_tensors(dev)
    torch.manual_seed(0)
    init = [ToyModel().flat_params.detach().clone() for _ in range(2)]
    tr = FusedTrainer(TOY_SPEC, 2, X, Y, SamplerGeometry(n=512, batch=256, seed=0), init_params=init)
    assert tr.groups == 4, tr.groups
    lib = nat.load()
    one(tr, lib, 20, "first")
    for _ in range(16):  # bench.py's warm-up launches
        tr.train(1)
    torch.cuda.synchronize()
    for i in range(5):
        one(tr, lib, 20, f"warm{i}")
    tr.close()


if __name__ == "__main__":
    main()
