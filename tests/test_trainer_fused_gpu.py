"""The Trainer trusts a LightningModule's fused_spec() only after checking it against
training_step on the first batch (trainer.py:_verify_fused_spec): an honest module runs
the fused engine, a module whose step differs from its declaration falls back to the
per-batch module path (or raises with engine="fused")."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from demo_pytorch_lightning import LitToyModel  # noqa: E402
from distributed_training_pytorch_amd.data.toy_data import ToyData  # noqa: E402
from distributed_training_pytorch_amd.trainer import Trainer  # noqa: E402


class GradLie(LitToyModel):
    """Logs the declared MSE, but trains model X on MSE plus an output penalty: same
    metric, another gradient direction (a plain rescale would be invisible to Adam)."""

    def training_step(self, batch, batch_idx, optimizer_idx=0):
        x, y = batch
        ox, oy = self(x)
        lx, ly = self.loss(ox, y), self.loss(oy, y)
        self.log("loss/lossX", lx)
        self.log("loss/lossY", ly)
        return lx + 0.5 * (ox ** 2).mean() + ly


class LossLie(LitToyModel):
    """Declares MSE but trains (and logs) an L1 loss."""

    def training_step(self, batch, batch_idx, optimizer_idx=0):
        x, y = batch
        ox, oy = self(x)
        lx, ly = torch.nn.functional.l1_loss(ox, y), torch.nn.functional.l1_loss(oy, y)
        self.log("loss/lossX", lx)
        self.log("loss/lossY", ly)
        return lx + ly


def _fit(model, tmp_path, engine="auto", steps=8):
    torch.manual_seed(0)
    dl = torch.utils.data.DataLoader(ToyData(seed=0), batch_size=128)
    tr = Trainer(gpus=1, max_steps=steps, accelerator="gpu", log_every_n_steps=1, default_root_dir=str(tmp_path),
                 enable_progress_bar=False, engine=engine)
    tr.fit(model, dl)
    return tr


def test_honest_fused_spec_runs_fused(tmp_path):
    torch.manual_seed(0)
    tr = _fit(LitToyModel(), tmp_path)
    assert tr.engine_used == "fused" and tr.fused_refused is None
    assert tr.global_step == 8


@pytest.mark.parametrize("cls,what", [(GradLie, "gradient"), (LossLie, "loss/lossX")])
def test_misdeclared_fused_spec_falls_back_to_module_path(tmp_path, cls, what):
    torch.manual_seed(0)
    lie = cls()
    torch.manual_seed(0)
    ref = LitToyModel()
    ref.load_state_dict(lie.state_dict())
    tr = _fit(lie, tmp_path / "lie")
    assert tr.engine_used == "module", tr.fused_refused
    assert tr.fused_refused and what in tr.fused_refused, tr.fused_refused
    assert tr.global_step == 8
    # the fallback trained what training_step computes, not the declaration: it ends
    # elsewhere than the honest module
    rtr = _fit(ref, tmp_path / "ref", engine="module")
    assert rtr.engine_used == "module"
    assert not torch.allclose(lie.model_X.flat_params, ref.model_X.flat_params)
    with pytest.raises(RuntimeError, match="fused"):
        _fit(cls(), tmp_path / "strict", engine="fused")
