"""Stock PyTorch-ROCm baseline arm (no framework kernels in the loop)."""
from .stock import StockBert, StockResNet50, run_stock  # noqa: F401
