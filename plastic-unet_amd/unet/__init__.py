from .unet_p import UNetp  # noqa: F401
from .unet_p_res import UNetpRes  # noqa: F401
from .coord_conv import CoordConvUNetp  # noqa: F401
