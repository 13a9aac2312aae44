"""TEST INFRASTRUCTURE ONLY - the CPU oracle for the plastic U-Net training path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this package, and only as the checker / the timed CPU baseline.  The product path
(``plastic-unet_amd/``) never imports it and fails loudly when its HIP library is missing.

The oracle is a plain PyTorch-CPU (fp32) restatement of yaricom/Plastic-UNet's math
(``src/unet/unet_p.py``, ``src/unet/unet_p_res.py``, ``src/train.py``, ``src/eval.py``,
``src/coord_conv_script.py``).  It is pinned against golden vectors generated from the reference
itself in the build container (``tests/golden/gen_golden.py`` -> ``tests/golden/*.npz``).
"""
from .ref_cpu import *  # noqa: F401,F403
