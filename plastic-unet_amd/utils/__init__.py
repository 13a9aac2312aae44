"""Host-side helpers of the eval/infer callers (numpy): the reference's IoU metric and RLE."""
from .iou_metric import fast_iou_metric, get_iou_vector  # noqa: F401
from .rle_encode import encode  # noqa: F401
