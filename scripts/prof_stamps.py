"""Phase breakdown of the fused train step from in-kernel s_memtime stamps.

Runs the diagnostic PROF instantiation (toy shape, Adam) for 8 iterations and
prints the cycles spent between stamps, per iteration, for wave 0 of model 0.
Stamp instrumentation costs cycles itself: read SHARES, not absolute length.
"""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_pytorch_amd import _native as nat  # noqa: E402
from distributed_training_pytorch_amd.data.sampler import SamplerGeometry  # noqa: E402
from distributed_training_pytorch_amd.data.toy_data import ToyData  # noqa: E402
from distributed_training_pytorch_amd.engine.fused_trainer import EngineConfig, FusedTrainer  # noqa: E402
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC  # noqa: E402

NAMES = ["step_start", "x_loaded", "fwd+loss", "bwd_done(w0)", "tiles_reduced", "grads_summed", "adam_done",
         "step_end"]


def main():
    # python scripts/prof_stamps.py [--lanes L --batch B]: L = 2 / 4 stamps the several-lanes step
    # --groups: the engine's split-batch step (csrc/grp_core.h; the default at batch > 64)
    lanes = int(sys.argv[sys.argv.index("--lanes") + 1]) if "--lanes" in sys.argv else 1
    batch = int(sys.argv[sys.argv.index("--batch") + 1]) if "--batch" in sys.argv else 256
    grouped = "--groups" in sys.argv
    dev = torch.device("cuda", 0)
    X, Y = ToyData(seed=0).device_tensors(dev)
    tr = FusedTrainer(TOY_SPEC, 2, X, Y, SamplerGeometry(n=512, batch=batch),
                      cfg=EngineConfig(groups="on" if grouped else "auto"))
    tr.train(50)  # warm
    tr.synchronize()
    lib = nat.load()
    nblk = 8 * max(1, tr.groups) if grouped else 2
    prof = torch.zeros(nblk * 8 * 32, dtype=torch.int64, device=dev)
    res = {}
    for rep in range(3):
        a = tr._train_args(8, nat.MODE_ADAM, None)
        a.status = nat.ptr(prof)
        if grouped:
            nat.check(lib.dtp_train_engine_profile(tr._engine_handle(), 8, tr.t, nat.ptr(prof), nat.stream_ptr()),
                      "engine profile")
        elif lanes > 1:
            nat.check(lib.dtp_mlp_train_profile_lanes(ctypes.byref(a), lanes, nat.stream_ptr()), "profile")
        else:
            nat.check(lib.dtp_mlp_train_profile(ctypes.byref(a), nat.stream_ptr()), "profile")
        torch.cuda.synchronize()
        st = prof.view(nblk, 8, 32).cpu()
        if grouped:  # per member of model 0 (blocks 0, 8, 16, ...): exchange = tiles_reduced -> grads_summed
            res.setdefault("members_exchange_cycles", []).append(
                [[int(st[8 * k, it, 5] - st[8 * k, it, 4]) for it in range(1, 8)] for k in range(tr.groups)])
            # inside the exchange (thread 0): tiles_reduced -> publish issued -> first poll consumed -> last
            # granule, polls; and each member's publish time relative to member 0's (skew)
            # XCC id and HW_ID (CU / SIMD / SE bits) of each member of model 0
            res.setdefault("placement", []).append([(int(st[8 * k, 0, 12]), hex(int(st[8 * k, 0, 13])))
                                                    for k in range(tr.groups)])
            # chip-wide s_memrealtime (10 ns ticks): each member's publish-issued and last-granule
            # times relative to the first member to publish (skew: the exchange waits for the last)
            for it in (3, 5):
                pubs = [int(st[8 * k, it, 14]) for k in range(tr.groups)]
                ends = [int(st[8 * k, it, 15]) for k in range(tr.groups)]
                p0 = min(pubs)
                res.setdefault("realtime_10ns", []).append({"publish": [p - p0 for p in pubs],
                                                             "last_granule": [e - p0 for e in ends]})
            res.setdefault("exchange_detail", []).append(
                [{"to_pub": int(st[8 * k, it, 16] - st[8 * k, it, 4]),
                  "pub_to_first_poll": int(st[8 * k, it, 17] - st[8 * k, it, 16]),
                  "pub_to_last": int(st[8 * k, it, 31] - st[8 * k, it, 16]),
                  "polls": int(st[8 * k, it, 30]),
                  "pub_skew_vs_m0": int(st[8 * k, it, 16] - st[0, it, 16])} for it in (3, 5) for k in range(tr.groups)])
        rows = []
        for it in range(1, 8):
            s = st[0, it]
            d = {NAMES[k]: int(s[k] - s[k - 1]) for k in range(1, 8)}
            d["total_step"] = int(st[0, it, 7] - st[0, it, 0]) if it else 0
            d["wave_bwd_end_rel"] = [int(st[0, it, 8 + w] - st[0, it, 0]) for w in range(4)]
            # layer-2 backward detail: staged (16), tile operands loaded (17), layer done (24+2)
            if int(st[0, it, 16]) and int(st[0, it, 17]):
                d["bwd_l2_detail"] = {"start->staged": int(st[0, it, 16] - st[0, it, 24 + 3]),
                                      "staged->tile_ops": int(st[0, it, 17] - st[0, it, 16]),
                                      "tile_ops->done": int(st[0, it, 24 + 2] - st[0, it, 17])}
            bl = [int(st[0, it, 24 + l]) for l in range(8) if int(st[0, it, 24 + l])][::-1]
            d["bwd_layers(top->0)"] = [int(b - a) for a, b in zip([int(s[2])] + bl[:-1], bl)]
            rows.append(d)
        res[rep] = rows[-1]
        # the launch's first step (cold instruction cache, LDS state just loaded)
        res[rep]["first_step_total"] = int(st[0, 0, 7] - st[0, 0, 0])
        # kernel entry -> first step start (parameter / dataset loads, weight scatter,
        # Adam table), and last step end -> write-back issued
        res[rep]["prologue"] = int(st[0, 0, 0] - st[0, 0, 20])
        res[rep]["epilogue"] = int(st[0, 0, 21] - st[0, 7, 7])
        # prologue detail (thread 0's view): dataset copied to LDS (18), first barrier
        # (19), weights scattered (22), Adam table filled (23), second barrier (29)
        marks = [("entry->data_copied", 20, 18), ("->barrier1", 18, 19), ("->weights_scattered", 19, 22),
                 ("->adam_table", 22, 23), ("->barrier2", 23, 29), ("->step0_start", 29, None)]
        res[rep]["prologue_detail"] = {name: int((st[0, 0, b] if b is not None else st[0, 0, 0]) - st[0, 0, a])
                                       for name, a, b in marks}
    print(json.dumps(res, indent=1))
    # also the wall time per step of the plain persistent kernel
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    tr.train(2000)
    ev1.record()
    torch.cuda.synchronize()
    print(json.dumps({"persistent_us_per_step": ev0.elapsed_time(ev1) * 1e3 / 2000, "engine_lanes": tr.lanes,
                      "batch": batch}))


if __name__ == "__main__":
    main()
