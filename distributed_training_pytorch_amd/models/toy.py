"""ToyModel: the reference's 5-layer LeakyReLU MLP (``toy_model_and_data.py:8-25``),
built for the fused HIP path.

* Same module tree and ``state_dict`` keys as the reference
  (``layers.{0,2,4,6,8}.{weight,bias}``), so checkpoints interchange.
* All parameters are views into ONE contiguous fp32 buffer (``flat_params``) in
  ``parameters()`` order -- the layout every kernel and the flat DDP all-reduce
  use.  The packing survives ``.to()/.cuda()`` (re-flattened in ``_apply``).
* On a CUDA input the forward is ONE fused kernel and the backward ONE fused
  kernel (``ops.mlp.FusedMLPFunction``); on CPU it is plain PyTorch.
* bf16 compute (``compute_dtype=torch.bfloat16`` or an enclosing
  ``torch.autocast(dtype=bfloat16)``): the bf16 instances of the same fused kernels
  (bf16 matmul operands, fp32 accumulation, fp32 master weights and gradients).
* Widths the fused kernel does not cover (hidden > 15) run every Linear on the
  MFMA GEMM with fused bias/LeakyReLU epilogues (``ops.gemm.mlp``), in fp32 or
  with bf16 compute.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops.gemm import mlp as gemm_mlp
from ..ops.mlp import MlpSpec, fused_mlp


class ToyModel(nn.Module):
    def __init__(self, in_features: int = 2, hidden: int = 10, depth: int = 3, out_features: int = 1,
                 slope: float = 0.01, compute_dtype: torch.dtype = torch.float32):
        super().__init__()
        self.spec = MlpSpec(in_features, hidden, depth + 2, out_features, False, slope)
        self.compute_dtype = compute_dtype
        self._fused: bool | None = None
        mods: list[nn.Module] = [nn.Linear(in_features, hidden), nn.LeakyReLU(slope)]
        for _ in range(depth):
            mods += [nn.Linear(hidden, hidden), nn.LeakyReLU(slope)]
        mods.append(nn.Linear(hidden, out_features))
        self.layers = nn.Sequential(*mods)
        self.flatten_parameters()

    # -- flat parameter packing ------------------------------------------------
    def flatten_parameters(self) -> torch.Tensor:
        ps = list(self.layers.parameters())
        if ps:
            flat = torch.empty(sum(p.numel() for p in ps), dtype=ps[0].dtype, device=ps[0].device)
            o = 0
            for p in ps:
                n = p.numel()
                flat[o:o + n].copy_(p.data.reshape(-1))
                p.data = flat[o:o + n].view_as(p)
                o += n
            self._flat = flat
        return self._flat

    def _packed(self) -> bool:
        """Are the parameters still consecutive views of ``_flat``?  Another owner (e.g.
        ``FlatDDP``) may have re-packed them into its own flat buffer."""
        ps = list(self.layers.parameters())
        base, es, o = self._flat.data_ptr(), self._flat.element_size(), 0
        for p in ps:
            if p.data_ptr() != base + o * es or not p.is_contiguous():
                return False
            o += p.numel()
        return o == self._flat.numel()

    @property
    def flat_params(self) -> torch.Tensor:
        """The parameters as one flat vector: the packed buffer itself, or -- once another
        owner re-packed the parameters -- a fresh concatenation of their current values."""
        if self._packed():
            return self._flat
        return torch.cat([p.detach().reshape(-1) for p in self.layers.parameters()])

    def _apply(self, fn, recurse=True):
        out = super()._apply(fn, recurse)
        self.flatten_parameters()
        return out

    def load_flat_(self, flat: torch.Tensor) -> None:
        with torch.no_grad():
            if self._packed():
                self._flat.copy_(flat.reshape(-1).to(self._flat))
                return
            o, flat = 0, flat.reshape(-1)
            for p in self.layers.parameters():  # re-packed elsewhere: write the live storage
                p.copy_(flat[o:o + p.numel()].view_as(p).to(p))
                o += p.numel()

    def uses_fused_kernel(self) -> bool:
        if self._fused is None:
            self._fused = self.compute_dtype == torch.float32 and self.spec.native_supported()
        return self._fused

    @staticmethod
    def forward_many(models: list["ToyModel"], x: torch.Tensor) -> tuple:
        """``tuple(m(x) for m in models)`` for ToyModels of one shape on the same input: on
        the GPU in fp32 (no autocast) the forwards run as ONE launch (``ops.mlp.
        fused_mlp_multi``), each backward its own launch; otherwise model by model."""
        ok = (x.is_cuda and len(models) > 1 and all(m.spec == models[0].spec for m in models)
              and not torch.is_autocast_enabled("cuda")
              and all(m.compute_dtype == torch.float32 and m.uses_fused_kernel() for m in models))
        if not ok:
            return tuple(m(x) for m in models)
        from ..ops.mlp import fused_mlp_multi

        return fused_mlp_multi(x.float(), models[0].spec, [list(m.layers.parameters()) for m in models])

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda:
            cd = self.compute_dtype
            if torch.is_autocast_enabled("cuda"):  # autocast (Trainer precision='bf16') picks the compute dtype
                cd = torch.get_autocast_dtype("cuda")
            if cd == torch.float32 and self.uses_fused_kernel():
                return fused_mlp(x.float(), self.spec, list(self.layers.parameters()))
            if cd == torch.bfloat16 and self.spec.native_supported(bf16=True):
                # fused stage kernels in bf16 compute: bf16 weights/activations, fp32
                # accumulation, fp32 master weights and gradients
                return fused_mlp(x.float(), self.spec, list(self.layers.parameters()), bf16=True)
            lin = [m for m in self.layers if isinstance(m, nn.Linear)]
            with torch.autocast("cuda", enabled=False):
                return gemm_mlp(x, [m.weight for m in lin], [m.bias for m in lin], self.spec.slope, cd)
        return self.layers(x)
