"""The README's "Using it with your own model" snippet runs as written (GPU)."""
import os
import re

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _snippet() -> str:
    text = open(os.path.join(ROOT, "README.md")).read()
    sec = text.split("## Using it with your own model", 1)[1]
    return re.search(r"```python\n(.*?)```", sec, re.S).group(1)


def test_readme_own_model_snippet(capsys):
    class MyModel(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.net = torch.nn.Sequential(torch.nn.Linear(2, 32), torch.nn.ReLU(), torch.nn.Linear(32, 1))

        def forward(self, x):
            return self.net(x)

    torch.manual_seed(0)
    v = torch.randn(512, 1, device="cuda")
    ns = {"MyModel": MyModel, "X": torch.cat([v, v], 1), "Y": v * v, "iters": 120, "world": 1, "rank": 0}
    exec(compile(_snippet(), "README.md", "exec"), ns)
    assert ns["stepper"].replays > 0
    lines = [l.split() for l in capsys.readouterr().out.splitlines() if l.strip()]
    assert len(lines) == 100  # two flushes of 50 steps
    first, last = float(lines[0][1]), float(lines[-1][1])
    assert last < first
