"""Layer-split model parallelism: K stages (+ GPipe micro-batches) must reproduce the
unsplit model's forward and gradients; CPU reference path and the fused GPU path
(stages co-located on cuda:0 when only one GPU is visible)."""
import pytest
import torch

from distributed_training_pytorch_amd.models.toy import ToyModel
from distributed_training_pytorch_amd.parallel.layer_split import LayerSplitMLP, default_boundaries


def _check(devs, bounds, mb, atol):
    torch.manual_seed(0)
    ref = ToyModel()
    x = torch.randn(96, 2)
    y = torch.randn(96, 1)
    ls = LayerSplitMLP(ref.spec, devs, bounds, mb, ref.flat_params.detach())
    out = ls(x)
    loss = torch.nn.functional.mse_loss(out, y.to(out.device))
    loss.backward()
    lr = torch.nn.functional.mse_loss(ref(x), y)
    lr.backward()
    torch.testing.assert_close(out.cpu(), ref(x).detach(), rtol=1e-5, atol=atol)
    g = torch.cat([p.grad.detach().cpu().reshape(-1) for p in ls.params])
    gr = torch.cat([p.grad.reshape(-1) for p in ref.parameters()])
    torch.testing.assert_close(g, gr, rtol=1e-4, atol=atol)


@pytest.mark.parametrize("K,mb", [(2, 1), (2, 4), (3, 1), (5, 3)])
def test_layer_split_cpu(K, mb):
    _check([torch.device("cpu")] * K, None, mb, 1e-6)


def test_boundaries():
    assert default_boundaries(5, 2) == [(0, 1), (2, 4)]
    assert default_boundaries(5, 3) == [(0, 1), (2, 3), (4, 4)]
    with pytest.raises(ValueError):
        default_boundaries(2, 3)


@pytest.mark.gpu
@pytest.mark.parametrize("K,mb", [(2, 1), (2, 4), (3, 2), (5, 1)])
def test_layer_split_gpu(K, mb):
    n = torch.cuda.device_count()
    devs = [torch.device("cuda", s % n) for s in range(K)]
    _check(devs, None, mb, 2e-5)
