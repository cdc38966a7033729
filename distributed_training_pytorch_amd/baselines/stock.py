"""Stock PyTorch-ROCm eager re-enactment of the reference's hot loop.

This is the comparison baseline of BASELINE.md ("reference semantics on stock
PyTorch-ROCm eager DDP (RCCL)"): plain nn.Sequential ToyModels (no fused
kernels), torch DDP, torch.optim.Adam, DistributedSampler + DataLoader(bs=256,
pin_memory=True), per-iteration ``.cpu()`` of both losses and a gloo
all-reduce of them -- the loop body of ``demo.py:95-129`` without wandb/tqdm.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
import torch.nn as nn
from torch.nn.parallel import DistributedDataParallel as DDP
from torch.utils.data import DataLoader, DistributedSampler


def plain_toy_model(slope: float = 0.01) -> nn.Module:
    return nn.Sequential(nn.Linear(2, 10), nn.LeakyReLU(slope), nn.Linear(10, 10), nn.LeakyReLU(slope),
                         nn.Linear(10, 10), nn.LeakyReLU(slope), nn.Linear(10, 10), nn.LeakyReLU(slope),
                         nn.Linear(10, 1))


class StockLoop:
    def __init__(self, dataset, device, batch: int = 256, seed: int = 0, ddp: bool = True):
        torch.manual_seed(seed)
        self.device = device
        self.mx = plain_toy_model().to(device)
        self.my = plain_toy_model().to(device)
        self.ddp = ddp and dist.is_initialized()
        if self.ddp:
            ids = [device.index] if device.type == "cuda" else None
            self.mx = DDP(self.mx, device_ids=ids)
            self.my = DDP(self.my, device_ids=ids)
        self.ox = torch.optim.Adam(self.mx.parameters(), lr=1e-3)
        self.oy = torch.optim.Adam(self.my.parameters(), lr=1e-3)
        self.sampler = DistributedSampler(dataset, shuffle=True) if dist.is_initialized() else None
        self.loader = DataLoader(dataset, batch_size=batch, sampler=self.sampler, shuffle=False,
                                 pin_memory=device.type == "cuda")
        self.gloo = dist.new_group(backend="gloo") if dist.is_initialized() else None
        self.world = dist.get_world_size() if dist.is_initialized() else 1
        self.loss = nn.MSELoss()
        self.epoch = 0
        self.it = None
        self.samples = 0
        self.last = (0.0, 0.0)

    def _next(self):
        while True:
            if self.it is None:
                if self.sampler is not None:
                    self.sampler.set_epoch(self.epoch)
                self.it = iter(self.loader)
            try:
                return next(self.it)
            except StopIteration:
                self.it = None
                self.epoch += 1

    def step(self):
        data, target = self._next()
        self.ox.zero_grad(set_to_none=True)
        self.oy.zero_grad(set_to_none=True)
        data = data.to(self.device)
        target = target.to(self.device)
        out_x = self.mx(data)
        out_y = self.my(data)
        lx = self.loss(out_x, target)
        lx.backward()
        ly = self.loss(out_y, target)
        ly.backward()
        self.ox.step()
        self.oy.step()
        b = target.size(0)
        rx = lx.detach().cpu() * b
        ry = ly.detach().cpu() * b
        if self.gloo is not None:
            dist.all_reduce(rx, group=self.gloo)
            dist.all_reduce(ry, group=self.gloo)
        self.last = (float(rx) / (b * self.world), float(ry) / (b * self.world))
        self.samples += b

    def train(self, n: int):
        for _ in range(n):
            self.step()

    def close(self):
        if self.gloo is not None:
            dist.destroy_process_group(self.gloo)
            self.gloo = None
