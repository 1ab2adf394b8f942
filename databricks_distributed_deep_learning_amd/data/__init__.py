"""Data loaders: synthetic ImageNet / token batches (Petastorm/Delta replacement)."""
from .synthetic import SyntheticImageNet, SyntheticTokens, shard_indices, IMAGENET_MEAN, IMAGENET_STD  # noqa: F401
from .transforms import resize, center_crop, normalize, to_tensor, imagenet_preprocess  # noqa: F401
