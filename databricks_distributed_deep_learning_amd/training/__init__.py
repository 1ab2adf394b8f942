"""Training loops (notebook-style ``train(cfg)``)."""
from .loop import Trainer, train  # noqa: F401
