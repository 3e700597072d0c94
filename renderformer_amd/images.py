"""Output image files of the reference CLIs (`infer.py:96-103`, `batch_infer.py:150-163`) without
imageio: HDR frames as OpenEXR (scanline, uncompressed, 32-bit float B/G/R channels — lossless
for the float32 render), LDR frames as 8-bit RGB PNG.  `read_exr` reads back the files written
here (tests)."""
from __future__ import annotations

import os
import struct
import zlib

import numpy as np

_EXR_MAGIC = 20000630
# zlib level of the PNG's IDAT stream: level 1 encodes a 512^2 frame ~6x faster than 6 (the file is ~20 % larger;
# the decoded pixels are identical); RF_PNG_LEVEL overrides
PNG_LEVEL = int(os.environ.get("RF_PNG_LEVEL", "1"))


def _attr(name: str, typ: str, data: bytes) -> bytes:
    return name.encode() + b"\0" + typ.encode() + b"\0" + struct.pack("<i", len(data)) + data


def write_exr(path: str, img: np.ndarray) -> None:
    """img: float [H, W, 3] (RGB) or [H, W] -> single-part scanline EXR, FLOAT pixels, no compression."""
    a = np.asarray(img, dtype=np.float32)
    if a.ndim == 2:
        a = a[..., None]
    if a.ndim != 3 or a.shape[2] not in (1, 3, 4):
        raise ValueError(f"write_exr: expected [H, W, 1|3|4], got {a.shape}")
    h, w, c = a.shape
    names = {1: ["Y"], 3: ["R", "G", "B"], 4: ["R", "G", "B", "A"]}[c]
    order = sorted(range(c), key=lambda i: names[i])  # EXR stores channels in name order
    chlist = b"".join(names[i].encode() + b"\0" + struct.pack("<iB3xii", 2, 0, 1, 1) for i in order) + b"\0"
    box = struct.pack("<iiii", 0, 0, w - 1, h - 1)
    header = struct.pack("<ii", _EXR_MAGIC, 2)
    header += _attr("channels", "chlist", chlist)
    header += _attr("compression", "compression", b"\0")
    header += _attr("dataWindow", "box2i", box)
    header += _attr("displayWindow", "box2i", box)
    header += _attr("lineOrder", "lineOrder", b"\0")
    header += _attr("pixelAspectRatio", "float", struct.pack("<f", 1.0))
    header += _attr("screenWindowCenter", "v2f", struct.pack("<ff", 0.0, 0.0))
    header += _attr("screenWindowWidth", "float", struct.pack("<f", 1.0))
    header += b"\0"
    line_bytes = w * c * 4
    start = len(header) + 8 * h
    offsets = (start + np.arange(h, dtype="<u8") * (8 + line_bytes)).astype("<u8")
    # every scanline as one record: int32 y, int32 byte count, then the [C, W] float32 planes of that line, so the
    # whole pixel block is one array and one write (per-line struct.pack + write was most of the file's time)
    lines = np.empty((h, 2 + c * w), dtype="<f4")
    lines_i = lines.view("<i4")
    lines_i[:, 0] = np.arange(h, dtype="<i4")
    lines_i[:, 1] = line_bytes
    lines[:, 2:] = a[:, :, order].transpose(0, 2, 1).reshape(h, c * w)  # [H, C, W]
    with open(path, "wb") as f:
        f.write(header)
        f.write(offsets.tobytes())
        f.write(lines.tobytes())


def read_exr(path: str) -> np.ndarray:
    """Reader for the files write_exr produces (uncompressed scanline FLOAT/HALF) -> [H, W, C] RGB order."""
    b = open(path, "rb").read()
    magic, _ = struct.unpack_from("<ii", b, 0)
    if magic != _EXR_MAGIC:
        raise ValueError("not an OpenEXR file")
    p = 8
    attrs = {}
    while b[p] != 0:
        e = b.index(b"\0", p)
        name = b[p:e].decode()
        e2 = b.index(b"\0", e + 1)
        size = struct.unpack_from("<i", b, e2 + 1)[0]
        attrs[name] = b[e2 + 5:e2 + 5 + size]
        p = e2 + 5 + size
    p += 1
    if attrs.get("compression", b"\0") != b"\0":
        raise ValueError("only uncompressed EXR is supported")
    ch, q = [], 0
    cl = attrs["channels"]
    while cl[q] != 0:
        e = cl.index(b"\0", q)
        ch.append((cl[q:e].decode(), struct.unpack_from("<i", cl, e + 1)[0]))
        q = e + 17
    x0, y0, x1, y1 = struct.unpack("<iiii", attrs["dataWindow"])
    w, h = x1 - x0 + 1, y1 - y0 + 1
    offs = struct.unpack_from(f"<{h}Q", b, p)
    out = np.zeros((h, len(ch), w), np.float32)
    for y, o in enumerate(offs):
        q = o + 8
        for ci, (_, pt) in enumerate(ch):
            dt, n = (np.dtype("<f4"), 4) if pt == 2 else (np.dtype("<f2"), 2)
            out[y, ci] = np.frombuffer(b, dtype=dt, count=w, offset=q)
            q += n * w
    names = [n for n, _ in ch]
    want = [n for n in ("R", "G", "B", "A", "Y") if n in names]
    return out.transpose(0, 2, 1)[:, :, [names.index(n) for n in want]]


def write_png(path: str, img: np.ndarray) -> None:
    """uint8 [H, W, 3] (or [H, W]) -> PNG (no filtering, zlib level 6)."""
    a = np.asarray(img)
    if a.dtype != np.uint8:
        raise ValueError("write_png expects uint8")
    if a.ndim == 2:
        a = a[..., None]
    h, w, c = a.shape
    ctype = {1: 0, 3: 2, 4: 6}[c]
    raw = b"".join(b"\0" + a[y].tobytes() for y in range(h))

    def chunk(tag: bytes, data: bytes) -> bytes:
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, ctype, 0, 0, 0))
    png += chunk(b"IDAT", zlib.compress(raw, PNG_LEVEL)) + chunk(b"IEND", b"")
    with open(path, "wb") as f:
        f.write(png)


def read_png(path: str) -> np.ndarray:
    """Reader for write_png output (8-bit, filter type 0 rows)."""
    b = open(path, "rb").read()
    p, idat, hdr = 8, b"", None
    while p < len(b):
        n = struct.unpack_from(">I", b, p)[0]
        tag = b[p + 4:p + 8]
        data = b[p + 8:p + 8 + n]
        if tag == b"IHDR":
            hdr = struct.unpack(">IIBBBBB", data)
        elif tag == b"IDAT":
            idat += data
        p += 12 + n
    w, h, _, ctype = hdr[:4]
    c = {0: 1, 2: 3, 6: 4}[ctype]
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + w * c)
    if (raw[:, 0] != 0).any():
        raise ValueError("read_png handles unfiltered rows only")
    return raw[:, 1:].reshape(h, w, c)


def hdr_to_ldr(hdr: np.ndarray) -> np.ndarray:
    """`infer.py:94-95` with tone_mapper 'none': clip to [0, 1], scale by 255, truncate to uint8."""
    return (np.clip(hdr, 0, 1) * 255).astype(np.uint8)
