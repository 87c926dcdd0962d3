"""Minimal PNG decoder for the tests: non-interlaced, colour types 0/2/3/4/6, bit depths 1-8,
all five row filters (lodepng picks the smallest encoding, e.g. 1-bit grey for a black frame).
Returns RGBA8 [h][w][4]."""
import struct
import zlib

import numpy as np

_CH = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}


def read_png(path):
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n", path
    pos, idat, plte, trns = 8, b"", None, None
    while pos < len(data):
        n, typ = struct.unpack(">I4s", data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        if typ == b"IHDR":
            w, h, depth, ctype, _, _, interlace = struct.unpack(">IIBBBBB", body)
            assert interlace == 0 and depth <= 8, (depth, interlace)
        elif typ == b"PLTE":
            plte = np.frombuffer(body, np.uint8).reshape(-1, 3)
        elif typ == b"tRNS":
            trns = body
        elif typ == b"IDAT":
            idat += body
        pos += 12 + n
    raw = zlib.decompress(idat)
    ch = _CH[ctype]
    stride = (w * ch * depth + 7) // 8
    bpp = max(1, ch * depth // 8)
    rows = np.zeros((h, stride), np.uint8)
    prev = np.zeros(stride, np.int32)
    for y in range(h):
        f = raw[y * (stride + 1)]
        line = np.frombuffer(raw, np.uint8, stride, y * (stride + 1) + 1).astype(np.int32)
        if f == 0:
            cur = line.copy()
        elif f == 2:
            cur = (line + prev) & 255
        else:
            cur = np.zeros(stride, np.int32)
            for x in range(stride):
                a = cur[x - bpp] if x >= bpp else 0
                b = prev[x]
                c = prev[x - bpp] if x >= bpp else 0
                if f == 1: p = a
                elif f == 3: p = (a + b) // 2
                else:
                    pa, pb, pc = abs(b - c), abs(a - c), abs(a + b - 2 * c)
                    p = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
                cur[x] = (line[x] + p) & 255
        rows[y] = cur
        prev = cur
    if depth < 8:
        bits = np.unpackbits(rows, axis=1)[:, :w * ch * depth].reshape(h, w * ch, depth)
        vals = (bits * (1 << np.arange(depth - 1, -1, -1))).sum(-1).astype(np.int32)
        if ctype != 3:
            vals = vals * 255 // ((1 << depth) - 1)
        samples = vals.reshape(h, w, ch)
    else:
        samples = rows[:, :w * ch].reshape(h, w, ch).astype(np.int32)
    out = np.full((h, w, 4), 255, np.uint8)
    if ctype == 3:
        out[..., :3] = plte[samples[..., 0]]
        if trns is not None:
            alpha = np.full(256, 255, np.uint8)
            alpha[:len(trns)] = np.frombuffer(trns, np.uint8)
            out[..., 3] = alpha[samples[..., 0]]
    elif ctype in (0, 4):
        out[..., 0] = out[..., 1] = out[..., 2] = samples[..., 0]
        if ctype == 4:
            out[..., 3] = samples[..., 1]
    else:
        out[..., :ch] = samples
    return out
