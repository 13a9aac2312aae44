"""Column-major run-length encoding of a binary mask (reference src/utils/rle_encode.py:6-17)."""
import numpy as np


def encode(im):
    pixels = np.concatenate([[0], np.asarray(im).flatten(order="F"), [0]])
    runs = np.where(pixels[1:] != pixels[:-1])[0] + 1
    runs[1::2] -= runs[::2]
    return " ".join(str(x) for x in runs)
