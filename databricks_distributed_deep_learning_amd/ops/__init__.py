"""Op layer: fused ops with HIP kernels on MI355X and PyTorch references on CPU.

Every public op dispatches per call:
  * GPU tensor + native library  -> hand-written HIP kernel (csrc/kernels/*.hip)
  * CPU tensor, or ``DDL_NATIVE=off`` -> plain PyTorch reference (also the
    numerical oracle the GPU tests compare against).

Layout conventions: images are NHWC (channels innermost so every channel run is
a 16-byte vector), conv weights are [Cout, KH, KW, Cin], linear weights are
[out, in] (PyTorch / HF convention).
"""
from ._lib import available as native_available, set_mode as set_native_mode, mode as native_mode  # noqa: F401
from ._lib import NativeUnavailable  # noqa: F401
from .conv import conv2d, conv2d_bias_act, patch_embed  # noqa: F401
from .norm import batch_norm, batch_norm_add_bn, bn_relu_maxpool, layer_norm  # noqa: F401
from .linear import linear  # noqa: F401
from .activation import gelu, dropout, relu  # noqa: F401
from .attention import attention  # noqa: F401
from .loss import cross_entropy, softmax_topk  # noqa: F401
from .pool import max_pool2d, global_avg_pool  # noqa: F401
from .embedding import embedding  # noqa: F401
from .glue import embedding_residual, first_token, prepend_token_add  # noqa: F401
