"""Lightning-style Module/Trainer (PL 1.5 semantics; pytorch_lightning itself is not required)."""
from .module import LightningModule  # noqa: F401
from .trainer import Trainer  # noqa: F401
