"""``Dataset.write_images`` (reference: python/ray/data/datasource/image_datasink.py)."""

from __future__ import annotations

import os

import numpy as np

import ray_amd as ray


@ray.remote
def _write_images_block(blk, path, column, file_format, idx):
    from PIL import Image

    os.makedirs(path, exist_ok=True)
    imgs = blk[column]
    for i in range(len(imgs)):
        Image.fromarray(np.asarray(imgs[i])).save(
            os.path.join(path, f"{idx:06d}_{i:06d}.{file_format}"))
    return len(imgs)
