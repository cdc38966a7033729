#!/usr/bin/env python3
"""The reference's model/data module (toy_model_and_data.py), MI355X edition.

``ToyModel`` keeps the reference's module tree and state_dict keys but runs its
forward and backward as fused HIP kernels on MI355X; ``ToyData`` draws the same
512-sample set (seeded, so every rank agrees unless ``per_rank=True``).
"""
from distributed_training_pytorch_amd.data.toy_data import ToyData  # noqa: F401
from distributed_training_pytorch_amd.models.toy import ToyModel  # noqa: F401

__all__ = ["ToyModel", "ToyData"]
