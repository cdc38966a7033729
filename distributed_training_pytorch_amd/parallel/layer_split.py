"""Layer-split (inter-layer) model parallelism with xGMI peer hand-off.

Reference: ``MultiGPUModel`` (``demo_one_model_multi_gpu.py:17-42``) puts
Linear(2,10)+Linear(10,10) on dev0 and the other three Linears on dev1, moves the
[B,10] activation with ``.to(dev1)`` and relies on autograd for the reverse copy;
DDP(device_ids=None) all-reduces per-device buckets.  There is no micro-batching.

MI355X design:
* K stages on K GPUs (any contiguous layer ranges, default = the reference split
  for K=2); each stage's forward is ONE fused kernel whose epilogue stores the
  activation directly into a buffer on the NEXT GPU (peer-mapped over xGMI, no
  separate memcpy); stage s's backward kernel reads its incoming gradient straight
  from stage s+1's GPU through the same peer mapping.  Cross-device ordering uses
  HIP events on the two devices' streams.
* optional GPipe micro-batching (``microbatches=M``): the host issues stage
  forwards in wavefront order so stage s works on micro-batch m while stage s+1
  works on m-1 (kernels on different devices run concurrently); autograd runs the
  backward per device thread, which pipelines the same way.
* data parallel on top: all stages' gradients of a process are packed into ONE
  flat buffer and all-reduced with a single collective (vs one bucket per device).
On CPU (or without the native library) stages fall back to PyTorch ops with the
same semantics.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn as nn

from .. import _native as nat
from ..ops.gemm import _fused_grad_target, _grad_ready, add_grad_ready_hook, mark_fused_grad
from ..ops.mlp import MlpSpec, mlp_forward_ref, stage_backward, stage_forward
from . import comm_util


def default_boundaries(n_layers: int, k: int) -> list[tuple[int, int]]:
    """Reference split for k=2 on the 5-layer toy (layers 0-1 | 2-4); else as even as possible."""
    if k == 2 and n_layers == 5:
        return [(0, 1), (2, 4)]
    base, rem = divmod(n_layers, k)
    out, a = [], 0
    for s in range(k):
        n = base + (1 if s < rem else 0)
        if n == 0:
            raise ValueError(f"cannot split {n_layers} layers over {k} stages")
        out.append((a, a + n - 1))
        a += n
    return out


def _enable_peer(a: torch.device, b: torch.device) -> None:
    if a.type != "cuda" or b.type != "cuda" or a == b:
        return
    import ctypes

    lib = nat.load()
    with torch.cuda.device(a):
        can = ctypes.c_int(0)
        nat.check(lib.dtp_can_access_peer(a.index, b.index, ctypes.byref(can)), "dtp_can_access_peer")
        if not can.value:
            raise RuntimeError(f"{a} cannot access {b} peer-to-peer")
        nat.check(lib.dtp_enable_peer_access(b.index), "dtp_enable_peer_access")


class _PeerStageFn(torch.autograd.Function):
    """One stage: fused forward on x.device whose epilogue also stores the output
    straight into a buffer on `dst` (peer store over xGMI); the backward kernel reads
    grad_out from `dst` through the same peer mapping (no staging copies)."""

    @staticmethod
    def forward(ctx, x, flat, spec: MlpSpec, dst: torch.device, force_peer: bool = False):
        src = x.device
        with torch.cuda.device(src):
            out, saved, out_dst = stage_forward(x, flat, spec, save=True, peer_device=dst, force_peer=force_peer)
            if dst != src:  # the consumer's stream waits for the producing kernel
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(src))
                torch.cuda.current_stream(dst).wait_event(ev)
        ctx.spec, ctx.src, ctx.dst = spec, src, dst
        ctx.param = flat  # the stage's Parameter: its persistent .grad takes the kernel's in-place add
        ctx.save_for_backward(x, flat, out, saved if saved is not None else torch.empty(0, device=src))
        return out_dst

    @staticmethod
    def backward(ctx, grad_out):
        x, flat, out, saved = ctx.saved_tensors
        src, dst = ctx.src, ctx.dst
        if dst != src:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(dst))
            torch.cuda.current_stream(src).wait_event(ev)
        # in place only into a persistent flat .grad the owner marked for it
        # (mark_fused_grad); anything else gets a fresh gradient through autograd,
        # so torch.autograd.grad and per-parameter hooks behave as usual
        g = _fused_grad_target(ctx.param) if ctx.needs_input_grad[1] else None
        inplace = g is not None and g.device == src
        with torch.cuda.device(src):
            gin, gp = stage_backward(x, flat, ctx.spec, out, saved if saved.numel() else None,
                                     grad_out.contiguous(), need_grad_in=ctx.needs_input_grad[0],
                                     grad_params=g if inplace else None)
            if dst != src:
                ev2 = torch.cuda.Event()
                ev2.record(torch.cuda.current_stream(src))
                torch.cuda.current_stream(dst).wait_event(ev2)
        if inplace:
            # the kernel already added into .grad: autograd has nothing to accumulate,
            # and the grad-ready hooks (per-stage DDP buckets) fire here instead
            _grad_ready(ctx.param)
            return gin, None, None, None, None
        return gin, gp, None, None, None


class LayerSplitMLP(nn.Module):
    def __init__(self, spec: MlpSpec, devices: list[torch.device], boundaries: list[tuple[int, int]] | None = None,
                 microbatches: int = 1, init_flat: torch.Tensor | None = None, force_peer_buffers: bool = False):
        super().__init__()
        # tests: hand activations over through the epilogue's second (peer) store even
        # between stages on the same GPU, as they are between distinct GPUs
        self.force_peer_buffers = force_peer_buffers
        self.spec = spec
        self.devices = [torch.device(d) for d in devices]
        self.boundaries = boundaries or default_boundaries(spec.n_layers, len(self.devices))
        if len(self.boundaries) != len(self.devices):
            raise ValueError("one layer range per device")
        self.microbatches = max(1, microbatches)
        if init_flat is None:
            from ..models.toy import ToyModel

            init_flat = ToyModel(spec.in_features, spec.hidden, spec.n_layers - 2, spec.out_features,
                                 spec.slope).flat_params.detach()
        self.stage_specs = [spec.substage(a, b) for a, b in self.boundaries]
        self.params = nn.ParameterList()
        for (a, b), dev in zip(self.boundaries, self.devices):
            lo, hi = spec.param_range(a, b)
            self.params.append(nn.Parameter(init_flat[lo:hi].detach().clone().to(dev)))
        for p in self.params:
            p.grad = torch.zeros_like(p)
            mark_fused_grad(p)  # the stage backward kernel adds into this persistent .grad
        for d0, d1 in zip(self.devices[:-1], self.devices[1:]):
            if d0.type == "cuda" and nat.native_enabled():
                _enable_peer(d0, d1)
                _enable_peer(d1, d0)

    @property
    def native(self) -> bool:
        return all(d.type == "cuda" for d in self.devices) and nat.native_enabled()

    def _stage(self, s: int, x: torch.Tensor, dst: torch.device) -> torch.Tensor:
        if self.native:
            return _PeerStageFn.apply(x, self.params[s], self.stage_specs[s], dst, self.force_peer_buffers)
        return mlp_forward_ref(self.params[s], self.stage_specs[s], x).to(dst)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = x.to(self.devices[0], non_blocking=True)
        K, M = len(self.devices), self.microbatches
        chunks = list(x.chunk(M)) if M > 1 else [x]
        M = len(chunks)
        acts = [[None] * (K + 1) for _ in range(M)]
        for m in range(M):
            acts[m][0] = chunks[m]
        # GPipe wavefront issue order: at tick t stage s runs micro-batch t - s
        for t in range(M + K - 1):
            for s in range(K):
                m = t - s
                if 0 <= m < M:
                    dst = self.devices[s + 1] if s + 1 < K else self.devices[s]
                    acts[m][s + 1] = self._stage(s, acts[m][s], dst)
        outs = [acts[m][K] for m in range(M)]
        return outs[0] if M == 1 else torch.cat(outs, 0)

    def flat_params_cpu(self) -> torch.Tensor:
        return torch.cat([p.detach().cpu() for p in self.params])

    def zero_grad(self, set_to_none: bool = False):
        for p in self.params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            else:
                p.grad.zero_()


class LayerSplitDDP:
    """Data parallel on top of a layer-split model, the way ``DDP(model,
    device_ids=None)`` treats a multi-device module (``demo_one_model_multi_gpu.py:
    96-98``): one gradient bucket PER DEVICE (per stage), each all-reduced as soon as
    that stage's backward has produced it -- from the stage parameter's grad-ready
    hook, on a side stream of the stage's own device -- so the last stage's bucket is
    on the wire while the earlier stages are still in their backward.

    Per bucket: the in-kernel xGMI one-shot all-reduce (``comm`` auto/xgmi, <= 8 ranks,
    buffers on the stage's device), RCCL (async work on the stage's device), or gloo
    (host-staged, CPU tests).  ``finish()`` (or the autograd end-of-backward callback)
    joins the streams; the averaging (1/W) is folded into the reduction."""

    def __init__(self, model: LayerSplitMLP, group=None, comm: str = "auto"):
        self.model = model
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.params = list(model.params)
        # construction broadcast of rank 0's parameters (per stage, on the stage's device)
        if self.world > 1:
            with torch.no_grad():
                for p in self.params:
                    comm_util.broadcast_(p.data, 0, group)
        self._xgmi: dict = {}
        self._side: dict = {}
        self.comm = "none" if self.world == 1 else ("gloo" if dist.get_backend(group) == "gloo" else "rccl")
        if self.world > 1 and comm in ("auto", "xgmi") and all(p.is_cuda for p in self.params):
            self._setup_xgmi(strict=comm == "xgmi")
        for p in self.params:
            p.register_post_accumulate_grad_hook(self._hook)
            add_grad_ready_hook(p, self._hook)
        self._pending: list = []
        self._queued = False
        self._done: set = set()
        self._fired = False  # a grad-ready hook fired since the last join

    def _setup_xgmi(self, strict: bool):
        from .xgmi import XgmiAllReduce

        ok, ars, why = True, {}, ""
        try:
            for i, p in enumerate(self.params):
                with torch.cuda.device(p.device):
                    ars[i] = XgmiAllReduce(p.numel(), p.device, self.group)
        except Exception as e:  # noqa: BLE001 - any mapping failure -> process-group buckets
            ok, why = False, str(e)
        flag = torch.tensor([1.0 if ok else 0.0])
        comm_util.all_reduce_(flag, self.group, op=dist.ReduceOp.MIN)
        if flag.item() == 1.0:
            self._xgmi = ars
            self._side = {i: torch.cuda.Stream(p.device) for i, p in enumerate(self.params)}
            self.comm = "xgmi"
            return
        for ar in ars.values():
            ar.close()
        if strict:
            raise RuntimeError(f"LayerSplitDDP comm='xgmi' unavailable: {why or 'a peer failed'}")

    def _hook(self, p):
        self._fired = True
        if not self._queued:
            torch.autograd.Variable._execution_engine.queue_callback(self.finish)
            self._queued = True
        i = next(k for k, q in enumerate(self.params) if q is p)
        if i in self._done:
            return
        self._done.add(i)
        self._reduce(i)

    def _reduce(self, i: int):
        if self.world == 1:
            return
        p = self.params[i]
        g = p.grad.view(-1)
        if i in self._xgmi:
            side = self._side[i]
            side.wait_stream(torch.cuda.current_stream(p.device))
            with torch.cuda.stream(side):
                self._xgmi[i].all_reduce_(g, scale=1.0 / self.world)
            self._pending.append(("xgmi", i))
        elif dist.get_backend(self.group) == "nccl":
            with torch.cuda.device(p.device):
                w = dist.all_reduce(g, group=self.group, async_op=True)
            self._pending.append((w, i))
        else:
            comm_util.all_reduce_(g, self.group)
            g.mul_(1.0 / self.world)
            self._pending.append((None, i))

    def finish(self):
        """Join every bucket's reduction; also the end-of-backward callback.  Idempotent:
        once a backward's buckets are joined, another call is a no-op until the next
        backward fires a grad hook (the demo calls it again after ``backward()``)."""
        if not self._fired and not self._pending:
            return
        if self._fired:
            for i in range(len(self.params)):  # stages that produced no gradient this backward
                if i not in self._done:
                    self._done.add(i)
                    self._reduce(i)
        for w, i in self._pending:
            p = self.params[i]
            if w == "xgmi":
                torch.cuda.current_stream(p.device).wait_stream(self._side[i])
            elif w is not None:
                w.wait()
                p.grad.mul_(1.0 / self.world)
        self._pending = []
        self._done = set()
        self._queued = False
        self._fired = False

    def allreduce_grads(self):
        """Reduce every stage's current ``.grad`` now, for callers that fill gradients
        without autograd (no grad hook fires); after a backward it only joins."""
        self._fired = True
        self.finish()

    def check_comm(self):
        for ar in self._xgmi.values():
            ar.check()

    def close(self):
        for ar in self._xgmi.values():
            ar.close()
        self._xgmi = {}


class FusedLayerSplit:
    """The layer-split model as persistent stage kernels (``csrc/split_train.hip``):
    stage s is ONE workgroup resident on ``devices[s]`` for every iteration of a
    ``train(k)`` call, sending its activation to stage s+1 and its input gradient to
    stage s-1 as epoch-tagged granules stored straight into the neighbour GPU's
    receive buffer (peer-mapped over xGMI), reducing its weight gradient over the
    data-parallel ranks in-kernel (per-device buckets, overlapped with the other
    stages' backward), with Adam / SGD fused.  The host issues one launch per stage
    per ``train(k)``; losses stay in a device ring on the last stage's GPU.

    Same semantics as the reference loop (``demo_one_model_multi_gpu.py:118-138``):
    forward through every stage, MSE on the last, backward, averaged gradients,
    one optimizer step per iteration; the sampler is the device DistributedSampler
    (``data/sampler.py``)."""

    def __init__(self, spec: MlpSpec, devices: list[torch.device], X: torch.Tensor, Y: torch.Tensor, geom,
                 optim, init_flat: torch.Tensor, boundaries: list[tuple[int, int]] | None = None, group=None,
                 timeout_us: int = 2_000_000, log_cap: int = 1 << 16, sampler: str = "torch",
                 launch: str = "per_device", members: int | str = "auto"):
        import ctypes

        from ..ops.optim import OptimConfig

        self.spec = spec
        self.devices = [torch.device(d) for d in devices]
        K = len(self.devices)
        self.bounds = boundaries or default_boundaries(spec.n_layers, K)
        self.stage_specs = [spec.substage(a, b) for a, b in self.bounds]
        self.optim = optim or OptimConfig()
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        if geom.world != self.world or geom.rank != self.rank:
            raise ValueError("sampler geometry does not match the process group")
        if geom.batch > 256:
            raise ValueError("the persistent split step runs one lane per sample: per-rank batch <= 256")
        self.geom = geom
        self.lib = lib = nat.require(self.devices[0])
        self.members = self._pick_members(members, lib, X, Y, geom)
        for s, ss in enumerate(self.stage_specs):
            if not lib.dtp_split_stage_supported(ss.in_features, ss.hidden, ss.n_layers, ss.out_features,
                                                 int(ss.final_act), int(s == 0)):
                raise NotImplementedError(f"no persistent split-stage kernel for stage {s}: {ss}")
        init = init_flat.detach().float().cpu().clone()
        if self.world > 1:  # DDP construction semantics: rank 0's weights everywhere
            comm_util.broadcast_(init, 0, group)
        for d0, d1 in zip(self.devices[:-1], self.devices[1:]):
            _enable_peer(d0, d1)
            _enable_peer(d1, d0)
        self.params, self.m, self.v, self.step, self.status = [], [], [], [], []
        for (a, b), dev in zip(self.bounds, self.devices):
            lo, hi = spec.param_range(a, b)
            self.params.append(init[lo:hi].to(dev))
            self.m.append(torch.zeros(hi - lo, device=dev))
            self.v.append(torch.zeros(hi - lo, device=dev))
            self.step.append(torch.zeros(1, dtype=torch.int32, device=dev))
            self.status.append(torch.zeros(16, dtype=torch.int32, device=dev))
        self.loss_log = torch.zeros(log_cap, device=self.devices[-1])
        self.X = X.to(self.devices[0]).contiguous().float()
        self.Y = Y.to(self.devices[-1]).contiguous().float()
        # link buffers: act into stage s+1 (on its device), grad into stage s (on its device).
        # Neighbours on one GPU talk through plain device memory at device scope (the
        # granules meet in the last-level cache); across GPUs through uncached fine-grained
        # buffers at system scope (xGMI).  DTP_SPLIT_LOCAL_LINKS=0 forces the latter (A/B).
        import os

        local_ok = os.environ.get("DTP_SPLIT_LOCAL_LINKS", "1") != "0"
        self._owned: list[tuple[int, int]] = []  # (device index, pointer)
        self._link_tensors: list[torch.Tensor] = []
        self.act_buf, self.grad_buf = [None] * K, [None] * K
        self.link_local = [local_ok and self.devices[s] == self.devices[s + 1] for s in range(K - 1)]
        for s in range(K - 1):
            width = self.stage_specs[s].out_features
            nbytes = int(lib.dtp_split_link_bytes(width, geom.batch))
            if self.link_local[s]:
                for buf in ("act", "grad"):
                    t = torch.zeros(nbytes, dtype=torch.uint8, device=self.devices[s])
                    self._link_tensors.append(t)
                    if buf == "act":
                        self.act_buf[s + 1] = t.data_ptr()
                    else:
                        self.grad_buf[s] = t.data_ptr()
            else:
                self.act_buf[s + 1] = self._alloc(self.devices[s + 1], nbytes)
                self.grad_buf[s] = self._alloc(self.devices[s], nbytes)
        # split-batch stages on one rank: each stage's on-chip member exchange buffer
        self._grp = [None] * K
        if self.members > 1 and self.world == 1:
            for s, (ss, dev) in enumerate(zip(self.stage_specs, self.devices)):
                nb = int(lib.dtp_split_lanes_grp_bytes(ss.P, self.members))
                self._grp[s] = torch.zeros(nb, dtype=torch.uint8, device=dev)
        # per-stage data-parallel exchange (the stage's gradient over the ranks)
        self._dp = [None] * K
        if self.world > 1:
            from .xgmi import PeerBuffers

            for s, (ss, dev) in enumerate(zip(self.stage_specs, self.devices)):
                with torch.cuda.device(dev):
                    self._dp[s] = PeerBuffers(int(lib.dtp_xgmi_fused_buffer_bytes(ss.P, 1, self.world)), dev, group)
        # sample order: the stages that gather (first: inputs, last: targets) read the
        # epoch permutations from a ring on their own GPU (torch's exact order by default)
        from ..data.sampler import SAMPLER_DIST_SHUFFLE, PermutationRing

        self.rings: dict = {}
        if geom.mode == SAMPLER_DIST_SHUFFLE:
            kind = "torch" if sampler == "torch" else "feistel"
            for dev in {self.devices[0], self.devices[-1]}:
                self.rings[dev] = PermutationRing(geom, dev, kind=kind)
        # launch = "per_device": the stages that share a GPU run as ONE launch (one
        # workgroup each: co-resident by construction), one stream per GPU.
        # launch = "per_stage": every stage is its own launch on its own stream -- what a
        # node with one GPU per stage runs anyway.  Stages that share a GPU then get
        # streams of DISTINCT priority levels, so no two of those persistent kernels (which
        # wait on each other) sit in one in-order hardware queue; this rehearses the
        # multi-GPU launch path on one GPU.  (CU-masked streams were tried first: they got
        # separate queues but dispatched one after the other, profiles/r4_split_streams/.)
        if launch not in ("per_device", "per_stage"):
            raise ValueError(f"launch={launch!r}: per_device or per_stage")
        self.launch_mode = launch
        self.groups: dict = {}  # launch key -> stage indices (key: device, or stage index)
        for s, dev in enumerate(self.devices):
            self.groups.setdefault(dev if launch == "per_device" else s, []).append(s)
        if any(len(v) > nat.SPLIT_MAX_LOCAL for v in self.groups.values()):
            raise ValueError(f"at most {nat.SPLIT_MAX_LOCAL} stages per GPU")
        self.key_dev = {k: self.devices[v[0]] for k, v in self.groups.items()}
        self.streams = {}
        for k, v in self.groups.items():
            dev = self.key_dev[k]
            on_dev = [s for s in range(K) if self.devices[s] == dev]
            if launch == "per_stage" and len(on_dev) > 1:
                levels = nat.stream_priority_levels(dev)
                if len(on_dev) > len(levels):
                    raise ValueError(f"launch='per_stage' with {len(on_dev)} stages on {dev}: only {len(levels)} "
                                     "stream priority levels; use launch='per_device'")
                self.streams[k] = nat.priority_stream(dev, levels[on_dev.index(v[0])])
            else:
                self.streams[k] = torch.cuda.Stream(device=dev)
        self.t = 0
        # devices whose split streams must wait for host-side state edits queued on the
        # current stream (construction synchronizes; load_state_dict / ring refills mark)
        self._dirty: set = set()
        self._copy_stream = None  # loss read-back, off the split streams' critical path
        self._copy_guards: list = []  # (event, first step) of the read-backs that may still read loss slots
        self._launch = {}
        for key, stages in self.groups.items():
            dev = self.key_dev[key]
            L = nat.SplitLaunch()
            L.n = len(stages)
            for j, s in enumerate(stages):
                ss = self.stage_specs[s]
                a = L.stage[j]
                a.X = nat.ptr(self.X) if s == 0 else None
                a.Y = nat.ptr(self.Y) if s == K - 1 else None
                a.params, a.opt_m, a.opt_v = nat.ptr(self.params[s]), nat.ptr(self.m[s]), nat.ptr(self.v[s])
                a.step, a.status = nat.ptr(self.step[s]), nat.ptr(self.status[s])
                a.loss_log = nat.ptr(self.loss_log) if s == K - 1 else None
                a.act_in = self.act_buf[s]
                a.act_out = self.act_buf[s + 1] if s + 1 < K else None
                a.grad_in = self.grad_buf[s]
                a.grad_out = self.grad_buf[s - 1] if s > 0 else None
                a.dp_peers = nat.ptr(self._dp[s].peer_table) if self._dp[s] is not None else None
                a.loss_log_cap = log_cap
                a.n_steps = 1
                a.timeout_us = int(timeout_us)
                a.cache_data = 1
                a.dp_world, a.dp_rank = self.world, self.rank
                a.optim = nat.MODE_ADAM if self.optim.name == "adam" else nat.MODE_SGD
                # bit 2: both ends of this stage's on-GPU links run in this launch, so their
                # members may switch to plain stores after the XCC hello (split_lanes.hip);
                # separate per-stage launches keep write-through links (measured faster there)
                same = all((s2 in stages) for s2 in (s - 1, s + 1) if 0 <= s2 < K)
                a.link_local = (int(s > 0 and self.link_local[s - 1])
                                | (int(s + 1 < K and self.link_local[s]) << 1) | (int(same) << 2))
                a.smp = geom.to_native()
                if dev in self.rings and (s == 0 or s == K - 1):
                    self.rings[dev].native(a.smp)
                a.hp = self.optim.hyper(spec.slope, 1.0 / self.world)
                a.grp_buf = nat.ptr(self._grp[s]) if self._grp[s] is not None else None
                L.shape_id[j] = lib.dtp_split_shape_id(ss.in_features, ss.hidden, ss.n_layers, ss.out_features,
                                                       int(ss.final_act), int(s == 0))
            L.members = self.members
            self._launch[key] = L
        self._launch_fn = lib.dtp_split_lanes_launch if self.members else lib.dtp_split_launch
        for d in set(self.devices):
            torch.cuda.synchronize(d)

    def _pick_members(self, members, lib, X, Y, geom) -> int:
        """Workgroups per stage of the split-batch stages (``csrc/split_lanes.hip``): each
        stage's per-rank batch over M members of <= 64 samples, member k of every stage one
        micro-batch flowing through the pipeline; 0 = the one-workgroup stages of
        ``split_train.hip``.  ``auto``: ceil(batch / 64) members wherever every stage has a
        split-batch instance (the toy model's layer ranges), the sampler reads the device
        permutation ring and the dataset fits the stages' LDS cache -- else 0.
        ``DTP_SPLIT_LANES=0`` forces 0 (A/B runs)."""
        import os

        if members in (0, "off") or os.environ.get("DTP_SPLIT_LANES", "1") == "0":
            return 0
        from ..data.sampler import SAMPLER_DIST_SHUFFLE

        K = len(self.stage_specs)
        ok = all(lib.dtp_split_lanes_supported(ss.in_features, ss.hidden, ss.n_layers, ss.out_features,
                                               int(ss.final_act), int(s == 0))
                 for s, ss in enumerate(self.stage_specs))
        ok = ok and geom.mode == SAMPLER_DIST_SHUFFLE
        ok = ok and geom.n * X.shape[1] <= 4096 and geom.n * Y.shape[1] <= 4096 and (K > 1 or
                                                                                  geom.n * (X.shape[1] + Y.shape[1]) <= 4096)
        need = -(-geom.batch // 64)
        if members == "auto":
            m = need
        else:
            m = int(members)
            if m < need:
                raise ValueError(f"members={m}: a member runs at most 64 samples (batch {geom.batch} needs >= {need})")
        if m * max(1, self.world) > 8 or m > 8 or m > geom.batch:
            if members != "auto":
                raise ValueError(f"members={m} x {self.world} ranks: the exchange serves at most 8")
            return 0
        if not ok:
            if members != "auto":
                raise ValueError("split-batch stages need the toy layer ranges, the device sampler ring and an "
                                 "LDS-sized dataset")
            return 0
        return m

    def _alloc(self, dev: torch.device, nbytes: int) -> int:
        import ctypes

        p = ctypes.c_void_p()
        with torch.cuda.device(dev):
            nat.check(self.lib.dtp_malloc_uncached(nbytes, ctypes.byref(p)), "dtp_malloc_uncached")
        self._owned.append((dev.index, p.value))
        return p.value

    def train(self, n_steps: int) -> None:
        """n_steps iterations: ONE persistent launch per GPU (its stages as co-resident
        workgroups), asynchronous.  Back-to-back calls queue on the split streams with no
        cross-stream wait unless something shared was rewritten in between."""
        if n_steps <= 0:
            return
        import ctypes

        for dev, ring in self.rings.items():
            e_lo, e_hi = ring.epochs_of_steps(self.t, self.t + n_steps - 1)
            keys = [k for k in self.streams if self.key_dev[k] == dev]
            if len(keys) == 1:
                # the one stream that reads this ring refills it too: stream order keeps
                # the copy behind the launches still reading the slots it overwrites
                with torch.cuda.stream(self.streams[keys[0]]):
                    ring.ensure(e_lo, e_hi)
            elif ring.needs_write(e_lo, e_hi):
                cur = torch.cuda.current_stream(dev)
                for k in keys:
                    cur.wait_stream(self.streams[k])
                ring.ensure(e_lo, e_hi)
                self._dirty.add(dev)
            else:
                ring.ensure(e_lo, e_hi)  # no copy; may start the next block's host generation
        last_key = self._last_key()
        cap = self.loss_log.shape[0]
        for key, L in self._launch.items():
            dev = self.key_dev[key]
            st = self.streams[key]
            if dev in self._dirty:
                st.wait_stream(torch.cuda.current_stream(dev))  # after the host-side state edits
            if key == last_key:
                self._copy_guards = [(ev, c0) for ev, c0 in self._copy_guards if not ev.query()]
                for ev, c0 in self._copy_guards:
                    if self.t + n_steps - c0 > cap:  # this launch's loss slots wrap onto unread ones
                        st.wait_event(ev)
            for j in range(L.n):
                L.stage[j].n_steps = n_steps
            with torch.cuda.device(dev):
                nat.check(self._launch_fn(ctypes.byref(L), nat.stream_ptr(st)), "dtp_split_launch")
        self._dirty.clear()
        self.t += n_steps

    def _last_key(self):
        """The launch that runs the last stage (it writes the loss log)."""
        return next(k for k, v in self.groups.items() if len(self.devices) - 1 in v)

    def _join(self):
        for k, st in self.streams.items():
            torch.cuda.current_stream(self.key_dev[k]).wait_stream(st)

    def synchronize(self):
        self._join()
        for d in set(self.devices):
            torch.cuda.synchronize(d)
        self.check_comm()

    def check_comm(self):
        self._join()
        for s, st in enumerate(self.status):
            w = st[:4].tolist()
            if w[0]:
                raise RuntimeError(f"layer-split link of stage {s} timed out at step {w[1] - 1} (neighbour stalled)")
            if w[2]:
                raise RuntimeError(f"data-parallel exchange of stage {s} timed out at step {w[3] - 1}")
        for s, st in enumerate(self.status):
            w = st[4:6].tolist()
            if w[0]:
                raise RuntimeError(f"member exchange of stage {s} timed out at step {w[1] - 1} (a member "
                                   "workgroup was not resident)")

    def losses(self, t0: int, t1: int) -> torch.Tensor:
        self._join()
        cap = self.loss_log.shape[0]
        t0 = max(t0, t1 - cap)
        ids = torch.arange(t0, t1) % cap
        return self.loss_log.index_select(0, ids.to(self.loss_log.device)).cpu()

    def losses_async(self, t0: int, t1: int):
        """Pinned copy of the losses of steps [t0, t1), queued on a copy stream behind the
        last stage's launch; ``.wait()`` returns [[loss], ...] (the fused engine's
        LossReadback).  The split streams never wait for it, unless a later launch's loss
        slots wrap onto the ones it still reads."""
        from ..engine.fused_trainer import LossReadback

        dev = self.devices[-1]
        if self._copy_stream is None:
            self._copy_stream = torch.cuda.Stream(device=dev)
        cs = self._copy_stream
        cs.wait_stream(self.streams[self._last_key()])
        cap = self.loss_log.shape[0]
        t0 = max(t0, t1 - cap)
        a, b = t0 % cap, t1 - t0
        with torch.cuda.device(dev), torch.cuda.stream(cs):
            src = (self.loss_log[a:a + b] if a + b <= cap
                   else torch.cat([self.loss_log[a:], self.loss_log[:a + b - cap]]))
            host = torch.empty(src.shape, pin_memory=True)
            host.copy_(src, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(cs)
        self._copy_guards.append((ev, t0))
        return LossReadback(host.view(-1, 1), None, ev, self.rank)

    def flat_params_cpu(self) -> torch.Tensor:
        self._join()
        return torch.cat([p.cpu() for p in self.params])

    def state_dict(self) -> dict:
        self._join()
        return {"params": self.flat_params_cpu(), "m": torch.cat([m.cpu() for m in self.m]),
                "v": torch.cat([v.cpu() for v in self.v]), "step": int(self.step[0].item()), "t": self.t}

    def load_state_dict(self, sd: dict) -> None:
        """Restore a checkpoint.  The link and data-parallel granules are tagged with the
        step number, so rewinding an engine that already trained past the checkpoint
        would let its receive buffers hand stale granules of later steps to the replay:
        that is refused (load into a freshly built engine instead)."""
        self._join()
        if int(sd["t"]) < self.t:
            raise RuntimeError(f"cannot rewind a layer-split engine from step {self.t} to {int(sd['t'])}: its "
                               "receive buffers hold granules of later steps; load into a fresh FusedLayerSplit")
        o = 0
        for s, p in enumerate(self.params):
            n = p.numel()
            p.copy_(sd["params"][o:o + n])
            self.m[s].copy_(sd["m"][o:o + n])
            self.v[s].copy_(sd["v"][o:o + n])
            self.step[s].fill_(int(sd["step"]))
            o += n
        self.t = int(sd["t"])
        self._dirty.update(self.devices)  # the next launches wait for these copies

    def close(self):
        import ctypes

        for s in range(len(self.devices)):
            torch.cuda.synchronize(self.devices[s])
        if self.world > 1 and dist.is_initialized():
            comm_util.barrier(self.group)  # no peer is still writing into our buffers
        for pb in self._dp:
            if pb is not None:
                pb.close()
        self._dp = [None] * len(self.devices)
        for dev_index, ptr in self._owned:
            with torch.cuda.device(dev_index):
                self.lib.dtp_free(ctypes.c_void_p(ptr))
        self._owned = []
        self._link_tensors = []
        for ring in getattr(self, "rings", {}).values():
            ring.close()  # its generator thread may be inside the native randperm
