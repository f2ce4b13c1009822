"""PNG files built in the tests (texture decoder parity): every colour type and bit depth, filter types cycling 0-4
per row, optionally Adam7-interlaced — layouts PIL does not write."""
import struct
import zlib

import numpy as np


def png_bytes(img, ctype, depth, interlace, palette=None):
    """A PNG file built here (zlib, filter types cycling 0-4 per row, optional Adam7 passes): img is (h, w, c) of
    sample values (uint8 or uint16)."""
    h, w = img.shape[:2]
    ch = img.shape[2]

    def pack(sub):
        rows = []
        bpp = max(1, ch * depth // 8)
        prev = bytes((sub.shape[1] * ch * depth + 7) // 8)
        for y in range(sub.shape[0]):
            if depth == 16:
                line = sub[y].astype(">u2").tobytes()
            elif depth == 8:
                line = sub[y].astype(np.uint8).tobytes()
            else:
                bits = "".join(format(int(v), f"0{depth}b") for v in sub[y].reshape(-1))
                bits += "0" * (-len(bits) % 8)
                line = bytes(int(bits[i:i + 8], 2) for i in range(0, len(bits), 8))
            ft = y % 5
            out = bytearray([ft])
            for i, v in enumerate(line):
                a = line[i - bpp] if i >= bpp else 0
                b = prev[i]
                c = prev[i - bpp] if i >= bpp else 0
                p0 = a + b - c
                pa, pb, pc = abs(p0 - a), abs(p0 - b), abs(p0 - c)
                paeth = a if pa <= pb and pa <= pc else (b if pb <= pc else c)
                out.append((v - (0, a, b, (a + b) // 2, paeth)[ft]) & 255)
            rows.append(bytes(out))
            prev = line
        return b"".join(rows)

    if interlace:
        passes = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]
        data = b"".join(pack(img[y0::dy, x0::dx]) for x0, y0, dx, dy in passes if img[y0::dy, x0::dx].size)
    else:
        data = pack(img)

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)

    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, depth, ctype, 0, 0, interlace))
    if palette is not None:
        png += chunk(b"PLTE", bytes(palette))
    return png + chunk(b"IDAT", zlib.compress(data, 6)) + chunk(b"IEND", b"")
