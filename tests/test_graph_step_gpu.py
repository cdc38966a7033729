"""engine/graph_step.py:CapturedStep on the GPU: warm-up, capture, replay per key, and
the eager fallback when a body cannot be captured."""
import pytest
import torch

from distributed_training_pytorch_amd.engine.graph_step import CapturedStep

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def test_captured_step_replays_per_key():
    acc = torch.zeros(4, device=DEV)
    inc = {2: torch.full((2,), 1.0, device=DEV), 4: torch.full((4,), 2.0, device=DEV)}

    def body(k):
        acc[:k].add_(inc[k])

    st = CapturedStep(body, DEV, warmup=2)
    for _ in range(5):
        st.run(2)
    for _ in range(3):
        st.run(4)
    torch.cuda.synchronize()
    # key 2: 2 eager warm-ups + capture-and-replay + 2 replays; key 4: 2 warm-ups + 1 replay
    assert st.is_captured(2) and st.is_captured(4) and st.replays == 4
    assert acc.tolist() == [5 + 6, 5 + 6, 6.0, 6.0]
    inc[2].fill_(10.0)  # static inputs are read at replay time
    st.run(2)
    torch.cuda.synchronize()
    assert acc[:2].tolist() == [21.0, 21.0]


def test_captured_step_falls_back_to_eager():
    acc = torch.zeros(1, device=DEV)
    aborted = []

    def body(_):
        acc.add_(1.0)
        if acc.item() < 0:  # a host sync: cannot be captured
            raise AssertionError

    st = CapturedStep(body, DEV, warmup=1, on_abort=lambda: aborted.append(1))
    for _ in range(4):
        st.run(None)
    torch.cuda.synchronize()
    assert not st.is_captured(None) and st.fallback_reason and aborted == [1]
    assert acc.item() == 4.0  # every iteration ran exactly once (the failed capture ran nothing)
