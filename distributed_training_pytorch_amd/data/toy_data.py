"""ToyData: the reference's synthetic regression set (``toy_model_and_data.py:27-36``).

512 samples, x = [v, v] with v ~ N(0, 1), y = v^2 + 0.5 * N(0, 1).  Drawn in the
reference's exact order (512 x ``randn``, then one ``randn(1)`` per sample) so a
seeded generator reproduces it bit for bit.  Unlike the reference (which is
unseeded, so every rank silently trains on a different dataset) the default
here is a seeded generator shared by all ranks; ``per_rank=True`` restores the
reference behaviour.

For the MI355X path the whole set is kept device resident (6 KB) and batches
are gathered in-kernel, replacing DataLoader collation + pinned H2D copies
(SURVEY.md §2.6 K13/K16).
"""
from __future__ import annotations

import torch
from torch.utils.data import Dataset


class ToyData(Dataset):
    def __init__(self, n: int = 512, seed: int | None = 0, rank: int = 0, per_rank: bool = False,
                 in_features: int = 2, classes: int = 0):
        g = torch.Generator()
        if seed is None:
            g.seed()
        else:
            g.manual_seed(int(seed) + (rank if per_rank else 0))
        v = torch.randn(n, generator=g)
        self.X = v.unsqueeze(1).repeat(1, in_features).contiguous()
        ys = [torch.randn(1, generator=g) * 0.5 + v[i] ** 2 for i in range(n)]
        self.Y = torch.stack(ys).reshape(n, 1).contiguous()
        if classes:
            # classification variant for the cross-entropy option: bucket y into classes
            edges = torch.quantile(self.Y.view(-1), torch.linspace(0, 1, classes + 1)[1:-1])
            self.Y = torch.bucketize(self.Y.view(-1), edges).float().view(n, 1)
        self.classes = classes

    def __getitem__(self, idx):
        return self.X[idx], self.Y[idx]

    def __len__(self):
        return self.X.shape[0]

    def device_tensors(self, device) -> tuple[torch.Tensor, torch.Tensor]:
        return self.X.to(device), self.Y.to(device)


def synthetic_toy(n: int, device, seed: int = 0) -> tuple[torch.Tensor, torch.Tensor]:
    """Fast vectorised variant (same distribution, different draw order) for large n."""
    g = torch.Generator().manual_seed(seed)
    v = torch.randn(n, generator=g)
    X = torch.stack([v, v], 1)
    Y = (v ** 2 + 0.5 * torch.randn(n, generator=g)).view(n, 1)
    return X.to(device), Y.to(device)
