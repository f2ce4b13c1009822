"""Writes the synthetic texture fixtures used by textures_mix.yaml (run from the repo root):
an RGB grid, a 4-bit palette image and an 8-bit grey ramp, so the product's PNG decoder sees
the colour types and filters the reference's image crate accepts."""
import os

import numpy as np
from PIL import Image

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "png")


def main():
    x, y = np.meshgrid(np.arange(48), np.arange(24))
    rgb = np.stack([(x * 5) % 256, (y * 10) % 256, (x * y * 7) % 256], axis=-1).astype(np.uint8)
    rgb[::6, :] = (250, 250, 250)
    rgb[:, ::8] = (20, 20, 20)
    Image.fromarray(rgb, "RGB").save(os.path.join(HERE, "tex_grid.png"))
    pal = Image.fromarray(((x[:8, :16] // 2 + y[:8, :16]) % 16).astype(np.uint8), "P")
    pal.putpalette([v for i in range(16) for v in (i * 16, 255 - i * 16, (i * 53) % 256)])
    pal.save(os.path.join(HERE, "tex_pal.png"), bits=4)
    grey = ((x[:10, :10] * 25 + y[:10, :10] * 3) % 256).astype(np.uint8)
    Image.fromarray(grey, "L").save(os.path.join(HERE, "tex_grey.png"))


if __name__ == "__main__":
    main()
