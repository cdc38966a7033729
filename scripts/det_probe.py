import os, sys, torch
sys.path.insert(0, os.getcwd())
from distributed_training_pytorch_amd.data.sampler import SamplerGeometry
from distributed_training_pytorch_amd.data.toy_data import ToyData
from distributed_training_pytorch_amd.engine.fused_trainer import EngineConfig, FusedTrainer
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC
from distributed_training_pytorch_amd.ops.optim import OptimConfig
dev = torch.device("cuda", 0)
X, Y = ToyData(n=512, seed=8).device_tensors(dev)
def run(spl, steps=19):
    g = torch.Generator().manual_seed(0)
    init = [(torch.randn(TOY_SPEC.P, generator=g) * 0.4).to(dev) for _ in range(2)]
    tr = FusedTrainer(TOY_SPEC, 2, X, Y, SamplerGeometry(n=512, batch=256, seed=4), OptimConfig(lr=1e-2),
                      EngineConfig(steps_per_launch=spl), init_params=init)
    tr.train(steps); tr.synchronize()
    r = tr.params.cpu().clone(), tr.losses(0, steps)
    tr.close(); return r
a = run(7); b = run(7); c = run(1); d = run(19)
for name, o in (("same", b), ("spl1", c), ("spl19", d)):
    print(name, (a[0]-o[0]).abs().max().item(), (a[1]-o[1]).abs().max().item(),
          [int(i) for i in ((a[1]-o[1]).abs().sum(1) > 0).nonzero().flatten()[:5]])
torch.save({"p": a[0], "l": a[1]}, f"gpurun_out/det_fast{os.environ.get('DTP_FAST','1')}.pt")
