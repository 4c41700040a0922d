"""Generates tests/golden/{cornell_box,cubes}_example.json from the reference's example renders
(/root/reference/examples/cornell_box.png and cubes.png, 600x450 RGBA; cornell_box.png was rendered
by the reference at 64 spp — render_examples.sh; cubes.png by an older build at a lower spp, SURVEY
§4). Only derived statistics are committed: the image mean and 30x30-pixel block means (20 x 15
blocks). Run in the build container (the reference is not on the GPU box)."""
import json
import os
import sys

import numpy as np
from PIL import Image

HERE = os.path.dirname(os.path.abspath(__file__))
SOURCES = {"cornell_box": "examples/cornell_box.png (reference, 600x450, 64 spp)",
           "cubes": "examples/cubes.png (reference, 600x450, older build, lower spp: qualitative pin, SURVEY 4)"}


def main():
    for name, note in SOURCES.items():
        im = np.asarray(Image.open(f"/root/reference/examples/{name}.png").convert("RGB")).astype(np.float64)
        h, w, _ = im.shape
        assert (w, h) == (600, 450)
        blocks = im.reshape(15, 30, 20, 30, 3).mean(axis=(1, 3))
        out = os.path.join(HERE, f"{name}_example.json")
        json.dump({"source": note, "width": w, "height": h, "image_mean": im.reshape(-1, 3).mean(0).round(4).tolist(),
                   "block": 30, "block_means": blocks.round(3).tolist()}, open(out, "w"))
        print("wrote", out)


if __name__ == "__main__":
    sys.exit(main())
