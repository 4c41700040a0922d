"""Generates tests/golden/cornell_box_example.json from the reference's example render
(/root/reference/examples/cornell_box.png, 600x450 RGBA, rendered by the reference at 64 spp —
render_examples.sh). Only derived statistics are committed: the image mean and 30x30-pixel block
means (20 x 15 blocks). Run in the build container (the reference is not on the GPU box)."""
import json
import os
import sys

import numpy as np
from PIL import Image

SRC = "/root/reference/examples/cornell_box.png"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cornell_box_example.json")


def main():
    im = np.asarray(Image.open(SRC).convert("RGB")).astype(np.float64)
    h, w, _ = im.shape
    assert (w, h) == (600, 450)
    blocks = im.reshape(15, 30, 20, 30, 3).mean(axis=(1, 3))
    json.dump({"source": "examples/cornell_box.png (reference, 600x450, 64 spp)", "width": w, "height": h,
               "image_mean": im.reshape(-1, 3).mean(0).round(4).tolist(),
               "block": 30, "block_means": blocks.round(3).tolist()}, open(OUT, "w"))
    print("wrote", OUT)


if __name__ == "__main__":
    sys.exit(main())
