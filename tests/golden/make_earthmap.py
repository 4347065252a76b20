"""Fixtures from the reference's texture input images/earthmap.jpg (used by its cuboidTest /
sphereUVTest demos and by demo2, test/Main.hs:117-137, 292):
  tests/golden/earthmap_128x64.npy  a 128 x 64 linear-RGB downsample, for the imageTexture tests;
  data/earthmap.png                 the full 1024 x 512 image's decoded 8-bit sRGB codes, stored
                                    losslessly (PNG), for scenes.demo2 (readImage linearises them).
The JPEG is decoded by Pillow; the reference decodes it with JuicyPixels (readImageAuto), whose
IDCT / chroma upsampling may differ from libjpeg's by a code here and there, so demo2's texture
is pinned to the file's content only up to that.

readImage (Ray.hs:241-245) decodes to `SRGB 'Linear` doubles, i.e. the sRGB transfer is undone;
this script does the same on a box-filtered 128 x 64 downsample and stores float16.
Run in the dev container (needs /root/reference and PIL); the .npy is committed."""
import os

import numpy as np
from PIL import Image

src = "/root/reference/images/earthmap.jpg"
codes = np.asarray(Image.open(src).convert("RGB"))
full = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "data", "earthmap.png")
Image.fromarray(codes).save(full, optimize=True)
print("wrote", full, codes.shape)
img = codes.astype(np.float64) / 255.0
lin = np.where(img <= 0.04045, img / 12.92, ((img + 0.055) / 1.055) ** 2.4)
h, w = lin.shape[:2]
lin = lin[: h - h % 64, : w - w % 128].reshape(64, (h - h % 64) // 64, 128, (w - w % 128) // 128, 3).mean((1, 3))
dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "earthmap_128x64.npy")
np.save(dst, lin.astype(np.float16))
print("wrote", dst, lin.shape, lin.mean((0, 1)))
