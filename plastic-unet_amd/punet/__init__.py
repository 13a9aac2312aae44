"""punet - host side of the MI355X plastic U-Net training path.

Layers: ``_lib`` (ctypes binding of libplastic_unet.so), ``kernels`` (tensor wrappers, one per C-ABI
entry point), ``trunk``/``head`` (autograd nodes that run only HIP kernels), ``optim`` (FusedAdam),
``dp`` (data parallel over RCCL), ``engine`` (the batched training step used by train.py/bench.py).
"""
from .head import BCELoss, bce_loss  # noqa: F401
from .optim import FusedAdam  # noqa: F401
