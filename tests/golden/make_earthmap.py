"""Fixture: a 128 x 64 linear-RGB copy of the reference's texture input images/earthmap.jpg
(used by its cuboidTest / sphereUVTest demos, test/Main.hs:117-137) for the imageTexture tests.

readImage (Ray.hs:241-245) decodes to `SRGB 'Linear` doubles, i.e. the sRGB transfer is undone;
this script does the same on a box-filtered 128 x 64 downsample and stores float16.
Run in the dev container (needs /root/reference and PIL); the .npy is committed."""
import os

import numpy as np
from PIL import Image

src = "/root/reference/images/earthmap.jpg"
img = np.asarray(Image.open(src).convert("RGB"), dtype=np.float64) / 255.0
lin = np.where(img <= 0.04045, img / 12.92, ((img + 0.055) / 1.055) ** 2.4)
h, w = lin.shape[:2]
lin = lin[: h - h % 64, : w - w % 128].reshape(64, (h - h % 64) // 64, 128, (w - w % 128) // 128, 3).mean((1, 3))
dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "earthmap_128x64.npy")
np.save(dst, lin.astype(np.float16))
print("wrote", dst, lin.shape, lin.mean((0, 1)))
