"""The Trainer demo's module-path helpers: several ToyModels on one input forward in ONE
launch (``ToyModel.forward_many`` -> ``ops.mlp.fused_mlp_multi``), against the models'
own fused forwards / backwards (bitwise), including a frozen model (the Trainer's
optimizer toggling) and the CPU fallback."""
import pytest
import torch

from distributed_training_pytorch_amd.models.toy import ToyModel


def test_forward_many_cpu_is_the_models_own():
    torch.manual_seed(0)
    ms = [ToyModel(), ToyModel()]
    x = torch.randn(16, 2)
    outs = ToyModel.forward_many(ms, x)
    for m, o in zip(ms, outs):
        assert torch.equal(o, m(x))


@pytest.mark.gpu
@pytest.mark.parametrize("freeze_second", [False, True])
def test_forward_many_matches_separate_fused_calls(freeze_second):
    torch.manual_seed(3)
    ms = [ToyModel().cuda(), ToyModel().cuda()]
    refs = [ToyModel().cuda(), ToyModel().cuda()]
    for r, m in zip(refs, ms):
        r.load_state_dict(m.state_dict())
    if freeze_second:
        for p in list(ms[1].parameters()) + list(refs[1].parameters()):
            p.requires_grad_(False)
    x = torch.randn(300, 2, device="cuda")  # two blocks of 256 per model
    y = torch.randn(300, 1, device="cuda")
    outs = ToyModel.forward_many(ms, x)
    assert "FusedMLPMulti" in type(outs[0].grad_fn).__name__
    routs = [r(x) for r in refs]
    for o, r in zip(outs, routs):
        assert torch.equal(o, r)
    loss = ((outs[0] - y) ** 2).mean() + ((outs[1] - y) ** 2).mean()
    rloss = ((routs[0] - y) ** 2).mean() + ((routs[1] - y) ** 2).mean()
    loss.backward()
    rloss.backward()
    for m, r in zip(ms, refs):
        for p, q in zip(m.parameters(), r.parameters()):
            if q.grad is None:
                assert p.grad is None
            else:
                assert torch.equal(p.grad, q.grad)
