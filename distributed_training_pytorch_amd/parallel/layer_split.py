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
from ..ops.gemm import _fused_grad_target, _grad_ready, mark_fused_grad
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
    def forward(ctx, x, flat, spec: MlpSpec, dst: torch.device):
        src = x.device
        with torch.cuda.device(src):
            out, saved, out_dst = stage_forward(x, flat, spec, save=True, peer_device=dst)
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
            return gin, None, None, None
        return gin, gp, None, None


class LayerSplitMLP(nn.Module):
    def __init__(self, spec: MlpSpec, devices: list[torch.device], boundaries: list[tuple[int, int]] | None = None,
                 microbatches: int = 1, init_flat: torch.Tensor | None = None):
        super().__init__()
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
            return _PeerStageFn.apply(x, self.params[s], self.stage_specs[s], dst)
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
    """Data parallel on top of a layer-split model: every stage's gradient is packed
    into one flat buffer on the first stage's device and all-reduced once."""

    def __init__(self, model: LayerSplitMLP, group=None):
        self.model = model
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        dev = model.devices[0]
        self.sizes = [p.numel() for p in model.params]
        self.buf = torch.zeros(sum(self.sizes), device=dev)
        if self.world > 1:  # construction broadcast of rank 0's parameters
            o = 0
            for p, n in zip(model.params, self.sizes):
                self.buf[o:o + n].copy_(p.detach().reshape(-1))
                o += n
            comm_util.broadcast_(self.buf, 0, group)
            o = 0
            with torch.no_grad():
                for p, n in zip(model.params, self.sizes):
                    p.copy_(self.buf[o:o + n].view_as(p))
                    o += n

    def allreduce_grads(self):
        if self.world == 1:
            return
        o = 0
        for p, n in zip(self.model.params, self.sizes):
            self.buf[o:o + n].copy_(p.grad.reshape(-1), non_blocking=True)
            o += n
        comm_util.all_reduce_(self.buf, self.group)
        self.buf.mul_(1.0 / self.world)
        o = 0
        for p, n in zip(self.model.params, self.sizes):
            p.grad.copy_(self.buf[o:o + n].view_as(p.grad), non_blocking=True)
            o += n
