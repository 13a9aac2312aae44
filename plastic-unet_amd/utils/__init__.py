"""Host-side helpers of the callers (numpy): the reference's IoU metric, RLE and the TGS loader."""
from .iou_metric import fast_iou_metric, get_iou_vector, iou_metric_batch  # noqa: F401
from .rle_encode import encode  # noqa: F401
from .data_set import load_train_dataset, load_test_dataset, load_image, cov_to_class  # noqa: F401
