"""Phase stamps of the fused split stage (diagnostic build: build.variant('splitprof',
['-DDTP_SPLIT_PROF=1'], ('split_train.hip',))); run with DTP_LIB pointing at it.
python scripts/split_stamps.py K -> per-step cycles between the LAST stage's phases."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_training_pytorch_amd.data.sampler import SamplerGeometry  # noqa: E402
from distributed_training_pytorch_amd.data.toy_data import ToyData  # noqa: E402
from distributed_training_pytorch_amd.ops.mlp import TOY_SPEC  # noqa: E402
from distributed_training_pytorch_amd.ops.optim import OptimConfig  # noqa: E402
from distributed_training_pytorch_amd.parallel.layer_split import FusedLayerSplit  # noqa: E402

NAMES = ["start", "x_ready", "fwd_done", "dz_ready", "bwd_done", "tiles_reduced", "grads_summed", "exchanged",
         "adam_done", "step_end"]

K = int(sys.argv[1]) if len(sys.argv) > 1 else 1
dev = torch.device("cuda", 0)
ds = ToyData(n=512, seed=2)
init = torch.randn(TOY_SPEC.P, generator=torch.Generator().manual_seed(0)) * 0.4
eng = FusedLayerSplit(TOY_SPEC, [dev] * K, ds.X, ds.Y, SamplerGeometry(n=512, batch=256, seed=1),
                      OptimConfig(lr=1e-3), init)
eng.train(20)
eng.synchronize()
eng.loss_log.zero_()
torch.cuda.synchronize(dev)  # the split streams do not wait on the current stream
eng.train(8)
eng.synchronize()
st = eng.loss_log[32768:32768 + 8 * 16 * 2].view(torch.int64).view(8, 16).cpu()
for it in range(2, 8):
    row = st[it]
    print(json.dumps({"K": K, "it": it, **{NAMES[k]: int(row[k] - row[k - 1]) for k in range(1, 10)},
                      "total": int(row[9] - row[0]), "to_next_start": int(st[it + 1][0] - row[0]) if it < 7 else None}))
eng.close()
