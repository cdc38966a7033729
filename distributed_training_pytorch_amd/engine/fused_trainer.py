"""FusedTrainer: the MI355X-native training engine for small MLP families.

One training iteration of the reference (``demo.py:95-129``: sampler ->
H2D -> fwd X, fwd Y -> MSE -> backward (DDP all-reduce) -> Adam x2 -> loss
all-reduce over gloo) becomes, per rank:

* ``comm="none"`` (W == 1):  ONE kernel launch for ``steps_per_launch``
  iterations of both models (persistent: weights, Adam state and the 6 KB
  dataset stay in LDS/registers), or a hipGraph of single-step launches.
* ``comm="rccl"``: fused grad kernel -> ``all_reduce`` of ONE flat buffer
  holding both models' gradients AND the two losses (RCCL over xGMI) ->
  fused flat-optimizer kernel.  Optionally captured into a hipGraph.
* ``comm="xgmi"``: ONE persistent kernel per ``steps_per_launch`` iterations;
  the all-reduce happens inside the step through peer-mapped xGMI buffers
  (``parallel/xgmi.py``).
* CPU tensors: the PyTorch reference of exactly the same step (gloo all-reduce).

The loss is never synchronised to the host inside the loop: every step writes
its global mean loss into a device ring (``loss_log``) read lazily.
"""
from __future__ import annotations

import ctypes
import math
import os
from dataclasses import dataclass, field

import torch
import torch.distributed as dist

from .. import _native as nat
from ..parallel import comm_util
from ..data.sampler import (SAMPLER_DIST_NOSHUFFLE, SAMPLER_DIST_SHUFFLE, SAMPLER_SEQUENTIAL, EpochIndexStream,
                             PermutationRing, SamplerGeometry)
from ..ops.mlp import MlpSpec, mlp_forward_ref
from ..ops.optim import OptimConfig, adam_update_ref, flat_optimizer_step, sgd_update_ref


@dataclass
class EngineConfig:
    comm: str = "auto"           # auto | none | rccl | xgmi | gloo
    launch: str = "persistent"   # persistent | graph | eager
    steps_per_launch: int = 1000  # persistent: iterations per kernel; graph: launches per graph
    # torch: the reference's exact DistributedSampler order (randperm(n) seeded with
    # seed+epoch), device: the keyed Feistel order; both read from a device ring of
    # upcoming epoch permutations (data/sampler.py: PermutationRing, SAMPLER_TABLE)
    sampler: str = "torch"
    loss: str = "mse"            # mse | ce
    log_cap: int = 1 << 16
    cache_data: bool = True
    xgmi_timeout_us: int = 2_000_000  # per exchange; sticky once hit (never multiplies over steps)
    xgmi_selftest: bool = True        # validate the xGMI exchange against a host all-reduce, else fall back
    rccl_graph: bool = True      # capture grad->all_reduce->optimizer into a hipGraph
    precision: str = "fp32"      # fp32 | bf16 (bf16 matmul operands, fp32 accumulation / master weights / Adam)
    # split-batch step (csrc/grp_core.h: a rank's batch over batch/64 workgroups per model):
    # auto = the measured policy (on for 4 members per model with several ranks), on, off
    groups: str = "auto"


class FusedTrainer:
    def __init__(self, spec: MlpSpec, n_models: int, X: torch.Tensor, Y: torch.Tensor,
                 geom: SamplerGeometry, optim: OptimConfig | None = None,
                 cfg: EngineConfig | None = None, init_params: list[torch.Tensor] | None = None,
                 group=None):
        self.spec = spec
        self.n_models = n_models
        self.optim = optim or OptimConfig()
        self.cfg = cfg or EngineConfig()
        if self.cfg.precision not in ("fp32", "bf16"):
            raise ValueError(f"precision {self.cfg.precision!r}: fp32 or bf16")
        self.geom = geom
        self.group = group
        self.device = X.device
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        if geom.world != self.world or geom.rank != self.rank:
            raise ValueError(f"sampler geometry ({geom.rank}/{geom.world}) does not match the process group "
                             f"({self.rank}/{self.world})")
        self.X = X.contiguous().float()
        self.Y = Y.contiguous().float()
        P = spec.P
        dev = self.device
        self.params = torch.empty(n_models, P, device=dev, dtype=torch.float32)
        if init_params is not None:
            for i, p in enumerate(init_params):
                self.params[i].copy_(p.reshape(-1))
        else:
            self.params.normal_(0, 0.3)
        self.m = torch.zeros_like(self.params)
        self.v = torch.zeros_like(self.params)
        self.step_ctr = torch.zeros(n_models, dtype=torch.int32, device=dev)
        self.loss_log = torch.zeros(self.cfg.log_cap, n_models, dtype=torch.float32, device=dev)
        self.comm_buf = torch.zeros(n_models * P + n_models, dtype=torch.float32, device=dev)
        self.t = 0  # host mirror of the step counter
        self._idx_stream = EpochIndexStream(geom)
        self._graphs: dict = {}
        self._engine = None  # native step executor (csrc/mlp_train.hip: dtp_train_engine_*)
        self._fast = None  # (run, engine, device, max steps, ring, steps/epoch): train()'s direct path
        self._dev_index = self.device.index if self.device.index is not None else (
            torch.cuda.current_device() if self.device.type == "cuda" else -1)
        self._xgmi = None
        self._ring = None
        self.comm_fallback_reason: str | None = None  # why an xGMI setup fell back to RCCL
        self.groups_refused: str | None = None  # why the split-batch step was not used
        self.comm = self._resolve_comm()
        # DDP construction semantics: every rank starts from rank 0's weights
        if self.world > 1:
            comm_util.broadcast_(self.params, 0, group)
        self.native = self.device.type == "cuda" and nat.native_enabled()
        if self.native:
            nat.require(self.device)
            if not spec.native_supported():
                raise NotImplementedError(f"no fused kernel for {spec}")
            lib = nat.require(self.device)
            if self.cfg.precision == "bf16" and not lib.dtp_mlp_train_bf16_supported(*spec.key[:4]):
                raise NotImplementedError(f"no bf16 fused train kernel for {spec}")
            ws = lib.dtp_mlp_workspace_floats(spec.in_features, spec.hidden, spec.n_layers, spec.out_features)
            if ws <= 0:
                raise NotImplementedError(f"no fused train kernel for {spec}")
            # scalar-weight workspace of the fused step (csrc/mlp_scalar.h), scratch
            self.wsp = torch.zeros(n_models * ws, dtype=torch.float32, device=dev)
            # Adam's per-step scalars, formed once on the host (f64, the kernels' own
            # arithmetic): a persistent launch loads them with its other prologue reads
            self._adam_tab = None
            if self.optim.name == "adam":
                from ..ops.optim import adam_bias_table

                tab = adam_bias_table(self.optim)
                if tab is not None:
                    self._adam_tab = torch.from_numpy(tab).to(dev)
            if geom.mode == SAMPLER_DIST_SHUFFLE:
                if self.cfg.sampler not in ("torch", "device"):
                    raise ValueError(f"sampler {self.cfg.sampler!r}: torch or device")
                self._ring = PermutationRing(geom, dev, kind="torch" if self.cfg.sampler == "torch" else "feistel")
            elif geom.mode == SAMPLER_DIST_NOSHUFFLE or (geom.mode == SAMPLER_SEQUENTIAL and geom.world == 1):
                # an unshuffled order as an identity table: the same indices, and the fast
                # step instances (which read a SAMPLER_TABLE ring) instead of the generic one
                self._ring = PermutationRing(geom, dev, kind="identity")
        if self.comm == "xgmi":
            self._setup_xgmi()

    @property
    def lanes(self) -> int:
        """Lanes per sample of the fused step instance this engine launches: 1 = the
        one-lane kernel, 2 / 4 = the several-lanes step (``csrc/mlp_lanes.h``) that the
        native dispatch picks for per-rank batches <= 128 / <= 64 (0: no fused kernel,
        e.g. a CPU engine or the RCCL path's grad kernel)."""
        return self._pick() & 0xFF

    @property
    def kernel_waves(self) -> int:
        """Waves per workgroup of the fused step instance (4: one per SIMD; 8: two, the
        several-lanes step over 512 / L samples); 0 without a fused kernel."""
        return (self._pick() >> 8) & 0xFF

    @property
    def groups(self) -> int:
        """Workgroups per model of the persistent step: > 1 is the split-batch step
        (``csrc/grp_core.h``: a rank's batch over several CUs per model, 64 samples each,
        their gradients summed on chip); 1 otherwise, 0 without a fused kernel."""
        return self._pick() >> 16

    def _pick(self) -> int:
        if not self.native or self.comm in ("rccl", "host"):
            return 0
        a = self._train_args(1, self._update_mode(), None)
        if self.groups_refused:
            a.groups = -1
        return int(nat.load().dtp_mlp_train_lanes(ctypes.byref(a), *self.spec.key[:4], self._update_mode()))

    # ------------------------------------------------------------------ setup
    def _resolve_comm(self) -> str:
        c = self.cfg.comm
        if self.device.type != "cuda":
            return "gloo" if self.world > 1 else "none"
        if c == "none" or (self.world == 1 and c == "auto"):
            if self.world > 1:
                raise ValueError("comm='none' with world > 1")
            return "none"
        if c == "auto":
            return "xgmi" if self.world <= 8 else "rccl"
        if c not in ("rccl", "xgmi", "host"):
            raise ValueError(f"comm {c!r} not valid for a GPU run with world={self.world}")
        if c == "xgmi" and self.world > 8:
            raise ValueError("comm='xgmi' is the single-node (<= 8 GPU) in-kernel exchange; use 'rccl' beyond")
        return c

    def _agree(self, ok: bool) -> bool:
        """True on every rank iff ``ok`` on every rank (one 1-element all-reduce)."""
        if self.world == 1:
            return ok
        flag = torch.tensor([0.0 if ok else 1.0], device="cpu")
        comm_util.all_reduce_(flag, self.group)
        return flag.item() == 0.0

    def _setup_xgmi(self):
        """Map the peers' exchange buffers; self-test; fall back to RCCL on any failure.

        Every collective here is issued by every rank whatever failed locally: the
        ranks agree on the setup before the self-test (whose first op is a
        collective), and again on its result, so a failure on some ranks only can
        never leave the others in a different collective."""
        from ..parallel.xgmi import XgmiExchange

        ok, why = True, ""
        try:
            self._xgmi = XgmiExchange(self.n_models, self.spec.P, self.device, self.group)
        except Exception as e:  # IPC / peer access unavailable
            ok, why = False, f"setup: {e}"
        ok = self._agree(ok)
        if ok and self.cfg.xgmi_selftest:
            ok, why = self._xgmi_selftest()
            ok = self._agree(ok)
        if not ok:
            self.comm_fallback_reason = why or "a peer failed the xGMI setup or self-test"
            if self.rank == 0:
                print(f"[dtp] xGMI exchange unavailable ({self.comm_fallback_reason}); using RCCL", flush=True)
            # the self-test's engine points at the peer buffers about to be unmapped: drop it
            # (and any graph captured on it) before the switch
            self._drop_engine()
            if self._xgmi is not None:
                if dist.is_initialized():
                    comm_util.barrier(self.group)
                self._xgmi.close()
                self._xgmi = None
            self.comm = "rccl"
            # the self-test restored every rank's state; re-broadcasting rank 0's
            # replica anyway makes the fallback safe by construction
            comm_util.broadcast_(self.params, 0, self.group)

    def _state(self):
        return (self.params, self.m, self.v, self.step_ctr, self.loss_log)

    def _xgmi_selftest(self) -> tuple[bool, str]:
        """Two exchanges (both buffer parities) of one real fused step through the
        in-kernel xGMI path must reproduce the host all-reduce path.  The training
        state is restored on every exit, and every rank issues the same collectives
        whatever fails locally."""
        import os

        lib = nat.load()
        saved = [t.clone() for t in self._state()]
        saved_t = self.t

        def restore():
            for t, s0 in zip(self._state(), saved):
                t.copy_(s0)

        try:
            ok, why = True, ""
            # reference: local grads via MODE_GRAD, host all-reduce, flat optimizer
            buf = torch.zeros_like(self.comm_buf)
            try:
                a = self._train_args(1, nat.MODE_GRAD, None)
                nat.check(lib.dtp_mlp_train(ctypes.byref(a), *self.spec.key[:4], nat.MODE_GRAD, nat.stream_ptr()),
                          "selftest grad")
                buf.copy_(self.comm_buf)
            except Exception as e:
                ok, why = False, f"selftest grad: {e}"
            comm_util.all_reduce_(buf, self.group)  # issued on every rank
            ok = self._agree(ok)
            if not ok:
                return False, why or "a peer failed the self-test"
            flat_optimizer_step(self.params, self.m, self.v, self.step_ctr, buf, self.optim,
                                grad_scale=1.0 / self.world, loss_log=self.loss_log, loss_scale=1.0 / self.world,
                                slope=self.spec.slope)
            ref_p = self.params.clone()
            ref_l = self.loss_log[0].clone()
            # the same step through the in-kernel exchange, twice (both parities); every
            # rank runs both launches (a rank that stopped early would leave its peers
            # waiting out the timeout); in-kernel waits are bounded
            errs = []
            for _ in range(2):
                restore()
                try:
                    self._run_engine(1)  # the engine's own instance (the split-batch step included)
                    torch.cuda.synchronize(self.device)
                except Exception as e:
                    errs.append(f"launch: {e}")
                    break
                st = self._xgmi.status[:2].tolist()
                if st[0]:
                    errs.append(f"timeout at epoch {st[1]}")
                    continue
                err = (self.params - ref_p).abs().max().item()
                lerr = (self.loss_log[0] - ref_l).abs().max().item()
                if not (err <= 1e-5 and lerr <= 1e-5):
                    errs.append(f"mismatch vs host all-reduce (param err {err:.3e}, loss err {lerr:.3e})")
            if os.environ.get("DTP_XGMI_SELFTEST_FAIL_RANK", "") == str(self.rank):
                errs.append("forced failure (DTP_XGMI_SELFTEST_FAIL_RANK)")  # test hook
            return (not errs), "; ".join(errs)
        except Exception as e:
            return False, f"selftest: {e}"
        finally:
            restore()
            self.t = saved_t

    def _hyper(self, grad_scale: float) -> nat.Hyper:
        return self.optim.hyper(self.spec.slope, grad_scale)

    def _train_args(self, n_steps: int, mode: int, idx: torch.Tensor | None, batch_override: int | None = None):
        g = self.geom
        smp = g.to_native()
        if self._ring is not None:
            self._ring.native(smp)
        if idx is not None:
            smp.mode = nat.SAMPLER_EXPLICIT
            smp.batch = batch_override or g.batch
        xg = self._xgmi
        a = nat.TrainArgs(
            nat.ptr(self.X), nat.ptr(self.Y), nat.ptr(idx), nat.ptr(self.params), nat.ptr(self.m), nat.ptr(self.v),
            nat.ptr(self.step_ctr), nat.ptr(self.comm_buf), nat.ptr(self.loss_log),
            nat.ptr(xg.status) if xg else None, nat.ptr(xg.peer_table) if xg else None,
            nat.ptr(xg.epoch) if xg else None, nat.ptr(getattr(self, "wsp", None)),
            self.loss_log.shape[0], self.n_models, n_steps,
            nat.LOSS_CE if self.cfg.loss == "ce" else nat.LOSS_MSE,
            int(self.cfg.cache_data), self.cfg.xgmi_timeout_us, int(self.cfg.precision == "bf16"), -1, smp,
            # xGMI modes sum the W gradients in-kernel -> DDP averaging 1/W there;
            # MODE_GRAD writes local means (the flat optimizer applies 1/W)
            self._hyper(1.0 / self.world if mode in (nat.MODE_XGMI_ADAM, nat.MODE_XGMI_SGD) else 1.0))
        tab = getattr(self, "_adam_tab", None)
        if tab is not None:
            a.adam_tab, a.adam_tab_len = nat.ptr(tab), tab.shape[0]
        if xg is not None:
            a.xbuf_bytes = xg.nbytes
        if self.cfg.groups not in ("auto", "on", "off"):
            raise ValueError(f"groups {self.cfg.groups!r}: auto, on or off")
        a.groups = {"auto": 0, "on": 1, "off": -1}[self.cfg.groups]
        return a

    def _update_mode(self) -> int:
        if self.comm == "xgmi":
            return nat.MODE_XGMI_ADAM if self.optim.name == "adam" else nat.MODE_XGMI_SGD
        return self.optim.kind

    # ------------------------------------------------------------------ steps
    def train(self, n_steps: int) -> None:
        """Run n_steps training iterations (asynchronous on the GPU)."""
        f = self._fast
        if f is not None and 0 < n_steps <= self.cfg.steps_per_launch:
            # the common call -- one persistent launch whose epochs are resident and far from
            # the ring's refill point -- straight to the native call (the general path's
            # Python bookkeeping is ~1.5 us of a 20-step call's ~85, scripts/launch_floor.py)
            run, e, di, _, ring, spe = f
            t = self.t
            if ring is None or ring.kind == "identity" or (
                    ring.lo <= t // spe and (t + n_steps) // spe <= ring.hi - (ring.E >> 1)):
                rc = run(e, n_steps, t, nat.raw_stream(di))
                if rc:
                    nat.check(rc, "dtp_train_engine_run")
                self.t = t + n_steps
                return
        if n_steps <= 0:
            return
        if not self.native:
            for _ in range(n_steps):
                self._reference_step()
            return
        if self.comm in ("rccl", "host"):
            remaining = n_steps
            G = max(1, min(self.cfg.steps_per_launch, 64))
            while remaining > 0:
                k = G if remaining >= G else 1
                self._ensure_epochs(k)
                self._rccl_steps(k)
                remaining -= k
            return
        remaining = n_steps
        while remaining > 0:
            if self.cfg.launch == "persistent":
                k = min(remaining, self.cfg.steps_per_launch)
                self._ensure_epochs(k)
                self._run_engine(k)
            elif self.cfg.launch == "graph":
                G = self.cfg.steps_per_launch
                if remaining >= G:
                    self._ensure_epochs(G)
                    self._graph_launch(G)
                    k = G
                else:  # a tail shorter than the captured graph: one-step launches via the native executor
                    k = 1
                    self._ensure_epochs(1)
                    self._run_engine(1)
            else:
                k = 1
                self._ensure_epochs(1)
                self._run_engine(1)
            remaining -= k
            self.t += k

    def _ensure_epochs(self, k: int) -> None:
        """The permutation ring holds every epoch the next k steps read (usually a no-op:
        the ring is filled ahead; a refill is one stream-ordered copy)."""
        if self._ring is not None:
            self._ring.ensure(*self._ring.epochs_of_steps(self.t, self.t + k - 1))

    def _drop_engine(self) -> None:
        """Destroy the native executor and every graph captured on it."""
        self._fast = None
        lib = nat.load() if self.native else None
        if self._engine is not None and lib is not None:
            lib.dtp_train_engine_destroy(self._engine)
        self._engine = None
        for h in list(self._graphs.values()):
            if isinstance(h, int) and lib is not None:
                lib.dtp_graph_destroy(ctypes.c_void_p(h))
        self._graphs.clear()

    def _engine_handle(self):
        """The native step executor (created once: argument block, kernel instance and, for
        the split-batch step, its on-chip exchange buffer)."""
        e = self._engine
        if e is None:
            lib = nat.load()
            mode = self._update_mode()
            a = self._train_args(1, mode, None)
            e = lib.dtp_train_engine_create(ctypes.byref(a), *self.spec.key[:4], mode)
            if not e:
                nat.check(-1, "dtp_train_engine_create")
            gr = lib.dtp_train_engine_groups(e)
            cus = nat.masked_stream_cus.get(nat.raw_stream(self._dev_index))
            if gr > 1 and cus is not None and cus < 8 * gr:
                # the split-batch members spin-wait on each other, so all 8 x groups
                # workgroups of its grid must be resident at once; a CU-masked stream with
                # fewer CUs (one workgroup per CU) would never dispatch some of them
                lib.dtp_train_engine_destroy(e)
                a.groups = -1
                e = lib.dtp_train_engine_create(ctypes.byref(a), *self.spec.key[:4], mode)
                if not e:
                    nat.check(-1, "dtp_train_engine_create")
                self.groups_refused = f"{cus} CUs on the masked stream < {8 * gr} split-batch workgroups"
            self._engine = e
            self._engine_run = lib.dtp_train_engine_run
            if (self.comm not in ("rccl", "host") and self.cfg.launch == "persistent"
                    and os.environ.get("DTP_TRAIN_FASTPATH", "1") != "0"):  # (=0: A/B)
                self._fast = (self._engine_run, e, self._dev_index, self.cfg.steps_per_launch, self._ring,
                              self.geom.steps_per_epoch)
        return e

    def _run_engine(self, k: int):
        """k iterations in one persistent launch through the native executor: the
        argument block is built once, so a call is one C call + one kernel launch."""
        e = self._engine_handle()
        # the host's step mirror (== the device counters) lets the kernel request its
        # first dataset indices without waiting for the counter load
        nat.check(self._engine_run(e, k, self.t, nat.raw_stream(self._dev_index)), "dtp_train_engine_run")

    def _launch(self, k: int, idx: torch.Tensor | None = None, batch_override: int | None = None):
        lib = nat.load()
        a = self._train_args(k, self._update_mode(), idx, batch_override)
        nat.check(lib.dtp_mlp_train(ctypes.byref(a), *self.spec.key[:4], self._update_mode(), nat.stream_ptr()),
                  "dtp_mlp_train")

    def _graph_launch(self, G: int):
        lib = nat.load()
        key = ("train", G)
        h = self._graphs.get(key)
        if h is None:
            # G one-step launches of the engine (the same kernel instance as the persistent
            # and eager launches -- the split-batch step included), each reading its step
            # number from the device counters so every replay continues
            e = self._engine_handle()
            s = torch.cuda.Stream(device=self.device)
            s.wait_stream(torch.cuda.current_stream())
            hp = ctypes.c_void_p()
            nat.check(lib.dtp_graph_capture_engine(e, G, nat.stream_ptr(s), ctypes.byref(hp)),
                      "dtp_graph_capture_engine")
            torch.cuda.current_stream().wait_stream(s)
            h = hp.value
            self._graphs[key] = h
        nat.check(lib.dtp_graph_launch(ctypes.c_void_p(h), nat.stream_ptr()), "dtp_graph_launch")

    def _rccl_steps(self, k: int):
        """k iterations of grad kernel -> RCCL all-reduce -> flat optimizer; with
        rccl_graph, all k captured in ONE hipGraph (one host replay per k steps: a
        replay costs ~10 us of host time, more than the step itself)."""
        lib = nat.load()
        if self.cfg.rccl_graph and self.comm == "rccl":
            g = self._graphs.get(("rccl", k))
            if g is None:
                g = self._capture_rccl(k)
            if g is not False:
                g.replay()
                self.t += k
                return
        for _ in range(k):
            self._rccl_body(lib)
            self.t += 1

    def _rccl_body(self, lib, idx=None, batch_override=None):
        a = self._train_args(1, nat.MODE_GRAD, idx, batch_override)
        nat.check(lib.dtp_mlp_train(ctypes.byref(a), *self.spec.key[:4], nat.MODE_GRAD, nat.stream_ptr()),
                  "dtp_mlp_train(grad)")
        comm_util.all_reduce_(self.comm_buf, self.group)
        flat_optimizer_step(self.params, self.m, self.v, self.step_ctr, self.comm_buf, self.optim,
                            grad_scale=1.0 / self.world, loss_log=self.loss_log, loss_scale=1.0 / self.world,
                            slope=self.spec.slope)

    def _capture_rccl(self, k: int = 1):
        lib = nat.load()
        try:
            s = torch.cuda.Stream(device=self.device)
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                # communicator warm-up on a scratch buffer (no training state touched)
                scratch = torch.zeros_like(self.comm_buf)
                comm_util.all_reduce_(scratch, self.group)
            s.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(k):
                    self._rccl_body(lib)
            torch.cuda.current_stream().wait_stream(s)
            self._graphs[("rccl", k)] = g
            return g
        except Exception as e:  # capture of collectives unsupported -> eager
            print(f"[dtp] hipGraph capture of the RCCL step failed ({e}); running eager", flush=True)
            self._graphs[("rccl", k)] = False
            return False

    # ------------------------------------------------------------------ CPU reference path
    def _reference_step(self):
        g = self.geom
        idx = torch.tensor(self._idx_stream.indices(self.t) if self.cfg.sampler == "torch" else g.indices(self.t),
                           dtype=torch.long, device=self.device)
        x, y = self.X[idx], self.Y[idx]
        grads = []
        losses = []
        for i in range(self.n_models):
            p = self.params[i].detach().clone().requires_grad_(True)
            out = mlp_forward_ref(p, self.spec, x)
            if self.cfg.loss == "ce":
                loss = torch.nn.functional.cross_entropy(out, y.view(-1).long())
            else:
                loss = torch.nn.functional.mse_loss(out, y.view_as(out))
            (gp,) = torch.autograd.grad(loss, p)
            grads.append(gp)
            losses.append(loss.detach().reshape(1))
        buf = torch.cat([torch.stack(grads).reshape(-1), torch.cat(losses)])
        if self.world > 1:
            comm_util.all_reduce_(buf, self.group)
        flat_optimizer_step(self.params, self.m, self.v, self.step_ctr, buf, self.optim,
                            grad_scale=1.0 / self.world, loss_log=self.loss_log, loss_scale=1.0 / self.world)
        self.t += 1

    # ------------------------------------------------------------------ state / logging
    def synchronize(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        self.check_comm()

    def step_indices(self, t: int) -> list[int]:
        """Dataset indices of this rank's batch at step t (the order the kernels read)."""
        return self._idx_stream.indices(t) if self.cfg.sampler == "torch" else self.geom.indices(t)

    def local_gradients(self) -> tuple[torch.Tensor, torch.Tensor]:
        """This rank's gradient [n_models, P] and mean loss [n_models] of the NEXT step
        (step ``t``'s batch, current weights), from the fused kernel's gradient-only launch
        (MODE_GRAD): no parameter, moment or step counter changes."""
        if not self.native:
            raise RuntimeError("local_gradients needs the native engine")
        self._ensure_epochs(1)
        lib = nat.load()
        a = self._train_args(1, nat.MODE_GRAD, None)
        a.host_t0 = self.t
        nat.check(lib.dtp_mlp_train(ctypes.byref(a), *self.spec.key[:4], nat.MODE_GRAD, nat.stream_ptr()),
                  "dtp_mlp_train(grad)")
        P, n = self.spec.P, self.n_models
        buf = self.comm_buf.clone()
        return buf[:n * P].view(n, P), buf[n * P:n * P + n]

    def exchange_stats_reset(self) -> None:
        """Zero the in-kernel exchange's wait / publish counters (status words [4..14),
        stream-ordered)."""
        if self._xgmi is not None:
            self._xgmi.status[4:14].zero_()

    def exchange_stats(self) -> tuple[float, int] | None:
        """(microseconds model 0's slowest thread spent between publishing its gradient
        granules and accepting its last peer granule, summed over the launches since the
        last reset; number of exchanges) -- None without the in-kernel xGMI exchange.
        Syncs."""
        st = self.exchange_stats_full()
        return None if st is None else (st["wait_us"], st["exchanges"])

    def exchange_stats_full(self) -> dict | None:
        """The exchange diagnostics since the last reset: ``wait_us`` (as exchange_stats),
        ``publish_us`` (the slowest publisher's first -> last granule store issued, summed
        over launches) and ``exchanges``.  None without the in-kernel xGMI exchange.  Syncs."""
        if self._xgmi is None:
            return None
        w = self._xgmi.status[4:14].cpu().view(torch.int64).tolist()
        # s_memrealtime runs at 100 MHz
        return {"wait_us": w[0] / 100.0, "exchanges": int(w[1]), "publish_us": w[3] / 100.0}

    def check_comm(self):
        """Raise if the in-kernel exchange (xGMI, or the split-batch step's on-chip one)
        hit its (sticky) timeout. One small read; call it where the host syncs anyway
        (loss readback, checkpoints)."""
        if self._xgmi is not None:
            self._xgmi.check_status()
        if self._engine is not None:
            st = (ctypes.c_int * 2)()
            nat.check(nat.load().dtp_train_engine_status(self._engine, st), "dtp_train_engine_status")
            if st[0]:
                raise RuntimeError(f"split-batch exchange timed out at epoch {st[1]} (a member workgroup was not "
                                   "resident)")

    def losses(self, t0: int, t1: int) -> torch.Tensor:
        """Global mean losses of steps [t0, t1) as a CPU tensor [t1-t0, n_models] (syncs)."""
        cap = self.loss_log.shape[0]
        if t1 - t0 > cap:
            t0 = t1 - cap
        ids = torch.arange(t0, t1) % cap
        return self.loss_log.index_select(0, ids.to(self.loss_log.device)).cpu()

    def losses_async(self, t0: int, t1: int) -> "LossReadback":
        """Queue a copy of the losses of steps [t0, t1) (and the xGMI status word) to
        pinned host memory behind the work already on the stream; ``.wait()`` returns
        them as a list of [n_models] rows without syncing on anything queued later."""
        cap = self.loss_log.shape[0]
        if t1 - t0 > cap:
            t0 = t1 - cap
        a, b = t0 % cap, t1 - t0
        if self.device.type != "cuda":
            rows = torch.cat([self.loss_log[a:], self.loss_log[:max(0, a + b - cap)]])[:b].clone()
            return LossReadback(rows, None, None, self.rank)
        src = self.loss_log[a:a + b] if a + b <= cap else torch.cat([self.loss_log[a:], self.loss_log[:a + b - cap]])
        host = torch.empty(src.shape, dtype=src.dtype, pin_memory=True)
        host.copy_(src, non_blocking=True)
        st = None
        if self._xgmi is not None:
            st = torch.empty(2, dtype=torch.int32, pin_memory=True)
            st.copy_(self._xgmi.status[:2], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        return LossReadback(host, st, ev, self.rank)

    def state_dict(self) -> dict:
        return {"params": self.params.detach().cpu(), "m": self.m.cpu(), "v": self.v.cpu(),
                "step": self.step_ctr.cpu(), "t": self.t, "spec": self.spec.__dict__,
                "optim": self.optim.__dict__}

    def load_state_dict(self, sd: dict):
        # the persistent launch takes its step number (sampler cursor AND Adam bias
        # corrections) from the host mirror t, so the device counters must equal it
        steps = torch.as_tensor(sd["step"]).reshape(-1).tolist()
        if any(int(s) != int(sd["t"]) for s in steps):
            raise ValueError(f"inconsistent engine state: step counters {steps} but t = {sd['t']}")
        self.params.copy_(sd["params"])
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        self.step_ctr.copy_(sd["step"])
        self.t = int(sd["t"])

    def model_params(self, i: int) -> torch.Tensor:
        return self.params[i]

    def close(self):
        self._drop_engine()
        if self._xgmi is not None:
            if dist.is_initialized():
                comm_util.barrier(self.group)
            self._xgmi.close()
            self._xgmi = None
        if self._ring is not None:
            self._ring.close()


class LossReadback:
    """Handle of :meth:`FusedTrainer.losses_async`."""

    def __init__(self, rows: torch.Tensor, status: torch.Tensor | None, event, rank: int):
        self.rows, self.status, self.event, self.rank = rows, status, event, rank

    def wait(self) -> list[list[float]]:
        return self.wait_tensor().tolist()

    def wait_tensor(self) -> torch.Tensor:
        """The rows as the host tensor they were copied into ([steps, n_models] fp32)."""
        if self.event is not None:
            self.event.synchronize()
        if self.status is not None and int(self.status[0]):
            raise RuntimeError(f"xGMI exchange timed out on rank {self.rank} at epoch {int(self.status[1])} "
                               "(peer not responding)")
        return self.rows
