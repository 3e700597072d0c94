"""Minimal HDF5 reader/writer for RenderFormer scene files, no h5py needed.

Scene files are written by the reference with h5py (`scene_processor/to_h5.py:87-92`):
five gzip-compressed datasets `triangles [N,3,3] f32`, `vn [N,3,3] f32`,
`texture [N,13,32,32] f16`, `c2w [V,4,4] f32`, `fov [V] f32` in the root group, read
back by `infer.py:12-30` / `batch_infer.py:27-58`.  This module restates the part of the
HDF5 file format those files use:

* superblock v0/v1 (h5py's default "earliest" format) and v2/v3;
* object headers v1 and v2 (with continuation blocks);
* old-style groups (symbol-table message -> v1 B-tree of SNOD nodes + local heap) and
  compact new-style groups (link messages);
* dataspace v1/v2, fixed-point / IEEE floating-point datatypes (either byte order, f16/f32/f64);
* layout message v1-v3: compact, contiguous and chunked (v1 B-tree chunk index) storage with
  the deflate (gzip) and shuffle filters.

Dense link storage (fractal heaps), layout v4 chunk indices, variable-length types and
attributes are not needed for scene files and raise ``H5FormatError``.  The writer emits
the same subset (superblock v0, v1 object headers, a symbol-table root group, chunked +
deflate datasets) so tests can build scene files; the reader is also checked against HDF5
files written by libhdf5 itself where such files exist on the machine (tests/test_h5io.py).
"""
from __future__ import annotations

import ctypes
import ctypes.util
import os
import struct
import threading
import time
import zlib
from typing import Dict, List, Optional, Tuple

import numpy as np

SIGNATURE = b"\x89HDF\r\n\x1a\n"
UNDEF = 0xFFFFFFFFFFFFFFFF


class H5FormatError(ValueError):
    pass


# ----------------------------------------------------------------------------------------- reader
_POOL = None
# callable(seconds) given the CPU time of every chunk decode (read + inflate + place), or None (batch_infer profiling)
CPU_HOOK = None


def host_threads() -> int:
    """CPU threads this process may use: the affinity mask, capped by a cgroup CPU quota (the GPU box shows 256
    CPUs and grants 16)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def _decode_pool():
    """Shared chunk-inflate pool (RF_H5_THREADS threads, default: every host thread, at most 16)."""
    global _POOL
    if _POOL is None:
        from concurrent.futures import ThreadPoolExecutor
        n = int(os.environ.get("RF_H5_THREADS", "0")) or min(16, host_threads())
        _POOL = ThreadPoolExecutor(max_workers=n, thread_name_prefix="h5inflate") if n > 1 else False
    return _POOL or None


_DEFLATE = None  # (libdeflate CDLL, per-thread decompressors) or False


def _libdeflate():
    """The system's libdeflate (ctypes; releases the GIL in the call), or None: inflates the scene texture's
    deflate chunks ~2-3x faster than zlib, straight into the destination array (no intermediate bytes).
    RF_H5_LIBDEFLATE=0 keeps zlib."""
    global _DEFLATE
    if _DEFLATE is None:
        _DEFLATE = False
        if os.environ.get("RF_H5_LIBDEFLATE", "1") != "0":
            try:
                lib = ctypes.CDLL(ctypes.util.find_library("deflate") or "libdeflate.so.0")
                lib.libdeflate_alloc_decompressor.restype = ctypes.c_void_p
                lib.libdeflate_alloc_decompressor.argtypes = []
                lib.libdeflate_free_decompressor.restype = None
                lib.libdeflate_free_decompressor.argtypes = [ctypes.c_void_p]
                lib.libdeflate_zlib_decompress.restype = ctypes.c_int
                lib.libdeflate_zlib_decompress.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t,
                                                           ctypes.c_void_p, ctypes.c_size_t,
                                                           ctypes.POINTER(ctypes.c_size_t)]
                _DEFLATE = (lib, threading.local())
            except (OSError, AttributeError):
                pass
    return _DEFLATE or None


class _Decompressor:
    """One thread's libdeflate decompressor (not thread-safe), freed with the thread's local storage."""

    def __init__(self, lib):
        self.lib, self.h = lib, lib.libdeflate_alloc_decompressor()

    def __del__(self):
        if self.h:
            self.lib.libdeflate_free_decompressor(self.h)
            self.h = None


def _inflate_into(raw: bytes, dst: np.ndarray) -> bool:
    """zlib-wrapped deflate stream `raw` decoded into the C-contiguous array `dst`, which it must fill exactly;
    False (nothing promised about dst) when libdeflate is absent or the stream does not decode to dst's size."""
    d = _libdeflate()
    if d is None:
        return False
    lib, tls = d
    dec = getattr(tls, "dec", None)
    if dec is None:
        dec = tls.dec = _Decompressor(lib)
    h = dec.h
    if not h:
        return False
    got = ctypes.c_size_t(0)
    rc = lib.libdeflate_zlib_decompress(h, raw, len(raw), dst.ctypes.data, dst.nbytes, ctypes.byref(got))
    return rc == 0 and got.value == dst.nbytes


class _Dataset:
    def __init__(self, f: "File", addr: int, msgs: List[Tuple[int, bytes]]):
        self._f = f
        self.shape: Tuple[int, ...] = ()
        self.dtype: Optional[np.dtype] = None
        self._layout = None
        self._filters: List[Tuple[int, Tuple[int, ...]]] = []
        for mtype, data in msgs:
            if mtype == 0x0001:
                self.shape = _parse_dataspace(data, f.sz_len)
            elif mtype == 0x0003:
                self.dtype = _parse_datatype(data)
            elif mtype == 0x0008:
                self._layout = _parse_layout(data, f.sz_off, f.sz_len)
            elif mtype == 0x000B:
                self._filters = _parse_filters(data)
        if self.dtype is None or self._layout is None:
            raise H5FormatError(f"object at {addr:#x} is not a dataset")

    def __array__(self, dtype=None, copy=None):
        a = self.read()
        return a.astype(dtype) if dtype is not None else a

    def read(self, out: Optional[np.ndarray] = None) -> np.ndarray:
        """The dataset as an array; with `out` (this shape and dtype, e.g. a view of a pinned host tensor) the data
        is decoded straight into it (batch_infer.py: no intermediate array, no copy into the pinned batch)."""
        kind = self._layout[0]
        n = int(np.prod(self.shape, dtype=np.int64)) if self.shape else 1
        nbytes = n * self.dtype.itemsize
        if out is not None and (tuple(out.shape) != tuple(self.shape) or out.dtype != self.dtype):
            raise ValueError(f"read(out=): expected {self.shape} {self.dtype}, got {tuple(out.shape)} {out.dtype}")
        if kind == "compact" or kind == "contiguous":
            if kind == "compact":
                raw = self._layout[1][:nbytes]
            elif self._layout[1] == UNDEF:
                raw = None
            else:
                raw = self._f._read(self._layout[1], nbytes)
            a = np.zeros(self.shape, dtype=self.dtype) if raw is None else \
                np.frombuffer(raw, dtype=self.dtype, count=n).reshape(self.shape)
            if out is None:
                return a.copy() if raw is not None else a
            out[...] = a
            return out
        # chunked: the file is read in order, the chunks are inflated in parallel (zlib releases the GIL; the
        # scene texture is ~90 % of a scene's decode time)
        btree, cdims = self._layout[1], self._layout[2]
        if btree == UNDEF:
            if out is None:
                return np.zeros(self.shape, dtype=self.dtype)
            out[...] = 0
            return out
        rank = len(self.shape)
        cshape = tuple(cdims[:rank])
        jobs, covered = [], 0
        for size, fmask, offs, caddr in self._f._chunk_entries(btree, rank):
            sl_out, sl_in, vol = [], [], 1
            for d in range(rank):
                lo = offs[d]
                hi = min(lo + cshape[d], self.shape[d])
                sl_out.append(slice(lo, hi))
                sl_in.append(slice(0, hi - lo))
                vol *= max(0, hi - lo)
            covered += vol
            jobs.append((self._f._read(caddr, size), fmask, tuple(sl_out), tuple(sl_in)))
        if out is None:
            out = (np.empty if covered == n else np.zeros)(self.shape, dtype=self.dtype)
        elif covered != n:
            out[...] = 0
        cn = int(np.prod(cshape))

        # deflate alone (the reference's gzip scene files): libdeflate straight into the chunk's slab of `out` when
        # the chunk is a whole C-contiguous piece of it, else into a chunk-sized scratch array
        inflate_only = [f[0] for f in self._filters] == [1]

        def place(job):
            raw, fmask, sl_out, sl_in = job
            if inflate_only and not fmask & 1:
                dst = out[sl_out]
                if dst.shape == cshape and dst.flags.c_contiguous:
                    if _inflate_into(raw, dst):
                        return
                else:
                    tmp = np.empty(cshape, dtype=self.dtype)
                    if _inflate_into(raw, tmp):
                        dst[...] = tmp[sl_in]
                        return
            raw = self._unfilter(raw, fmask)
            out[sl_out] = np.frombuffer(raw, dtype=self.dtype, count=cn).reshape(cshape)[sl_in]
        if CPU_HOOK is not None:  # profiling (batch_infer RF_BATCH_PROFILE): CPU seconds of the chunk decode threads
            plain = place

            def place(j):
                t0 = time.thread_time()
                try:
                    plain(j)
                finally:
                    CPU_HOOK(time.thread_time() - t0)
        pool = _decode_pool() if len(jobs) > 1 else None
        if pool is None:
            for j in jobs:
                place(j)
        else:
            list(pool.map(place, jobs))
        return out

    def _unfilter(self, raw: bytes, fmask: int) -> bytes:
        for i in reversed(range(len(self._filters))):
            fid, cd = self._filters[i]
            if fmask & (1 << i):
                continue  # filter skipped for this chunk
            if fid == 1:
                raw = zlib.decompress(raw)
            elif fid == 2:
                size = cd[0] if cd else self.dtype.itemsize
                a = np.frombuffer(raw, dtype=np.uint8)
                ne = a.size // size
                body = a[: ne * size].reshape(size, ne).T.reshape(-1)
                raw = body.tobytes() + a[ne * size:].tobytes()
            elif fid == 3:
                raw = raw[:-4]  # fletcher32 checksum trailer
            else:
                raise H5FormatError(f"unsupported filter id {fid}")
        return raw


class File:
    """Read-only HDF5 file: ``File(path)['triangles']`` -> dataset; ``np.array(ds)`` reads it."""

    def __init__(self, path: str, mode: str = "r"):
        if mode != "r":
            raise ValueError("h5io.File is read-only; use write_datasets() to create files")
        with open(path, "rb") as fh:
            self._buf = fh.read()
        self.path = path
        base = self._find_superblock()
        b = self._buf
        ver = b[base + 8]
        if ver in (0, 1):
            self.sz_off, self.sz_len = b[base + 13], b[base + 14]
            p = base + 24 + (4 if ver == 1 else 0)
            self.base = self._uint(p, self.sz_off)
            p += 4 * self.sz_off  # base, free-space, EOF, driver info
            # root symbol-table entry: name offset, object header address, cache type, reserved, scratch
            root = self._uint(p + self.sz_off, self.sz_off)
        elif ver in (2, 3):
            self.sz_off, self.sz_len = b[base + 9], b[base + 10]
            p = base + 12
            self.base = self._uint(p, self.sz_off)
            root = self._uint(p + 3 * self.sz_off, self.sz_off)
        else:
            raise H5FormatError(f"unsupported superblock version {ver}")
        self._root = self._group_links(root)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def close(self):
        self._buf = b""

    def keys(self):
        return list(self._root.keys())

    def __contains__(self, name):
        return name in self._root

    def __getitem__(self, name: str) -> _Dataset:
        links = self._root
        parts = [p for p in name.split("/") if p]
        for i, part in enumerate(parts):
            if part not in links:
                raise KeyError(name)
            addr = links[part]
            msgs = self._object_messages(addr)
            if i < len(parts) - 1:
                links = self._links_from_messages(msgs)
            else:
                if any(t in (0x0011, 0x0006, 0x0002) for t, _ in msgs) and not any(t == 0x0008 for t, _ in msgs):
                    raise KeyError(f"{name} is a group")
                return _Dataset(self, addr, msgs)
        raise KeyError(name)

    # -- primitives
    def _find_superblock(self) -> int:
        off = 0
        while off < len(self._buf):
            if self._buf[off:off + 8] == SIGNATURE:
                return off
            off = 512 if off == 0 else off * 2
        raise H5FormatError("not an HDF5 file")

    def _uint(self, p: int, n: int) -> int:
        return int.from_bytes(self._buf[p:p + n], "little")

    def _read(self, addr: int, n: int) -> bytes:
        p = self.base + addr
        if p + n > len(self._buf):
            raise H5FormatError("read past end of file")
        return self._buf[p:p + n]

    # -- object headers
    def _object_messages(self, addr: int) -> List[Tuple[int, bytes]]:
        p = self.base + addr
        b = self._buf
        if addr == UNDEF or p + 16 > len(b):
            raise H5FormatError(f"object header address {addr:#x} outside the file")
        msgs: List[Tuple[int, bytes]] = []
        if b[p:p + 4] == b"OHDR":
            flags = b[p + 5]
            q = p + 6
            if flags & 0x20:
                q += 16
            if flags & 0x10:
                q += 4
            nsz = 1 << (flags & 3)
            size0 = self._uint(q, nsz)
            q += nsz
            blocks = [(q, size0)]
            while blocks:
                start, size = blocks.pop(0)
                q, end = start, start + size
                while q + 4 <= end:
                    mtype, msize, mflags = b[q], self._uint(q + 1, 2), b[q + 3]
                    q += 4 + (2 if flags & 0x04 else 0)
                    data = b[q:q + msize]
                    q += msize
                    if mtype == 0x10:
                        caddr, clen = self._uint(q - msize, self.sz_off), self._uint(q - msize + self.sz_off, self.sz_len)
                        blocks.append((self.base + caddr + 4, clen - 8))  # skip "OCHK", checksum
                    elif mtype != 0:
                        msgs.append((mtype, data))
            return msgs
        if b[p] != 1:
            raise H5FormatError(f"unsupported object header version {b[p]} at {addr:#x}")
        nmsgs = self._uint(p + 2, 2)
        hsize = self._uint(p + 8, 4)
        blocks = [(p + 16, hsize)]
        while blocks and len(msgs) < nmsgs + 64:
            start, size = blocks.pop(0)
            q, end = start, start + size
            while q + 8 <= end:
                mtype, msize = self._uint(q, 2), self._uint(q + 2, 2)
                data = b[q + 8:q + 8 + msize]
                q += 8 + msize
                if mtype == 0x10:
                    blocks.append((self.base + int.from_bytes(data[:self.sz_off], "little"),
                                   int.from_bytes(data[self.sz_off:self.sz_off + self.sz_len], "little")))
                elif mtype != 0:
                    msgs.append((mtype, data))
        return msgs

    # -- groups
    def _group_links(self, addr: int) -> Dict[str, int]:
        return self._links_from_messages(self._object_messages(addr))

    def _links_from_messages(self, msgs) -> Dict[str, int]:
        links: Dict[str, int] = {}
        for mtype, data in msgs:
            if mtype == 0x0011:
                btree = int.from_bytes(data[:self.sz_off], "little")
                heap = int.from_bytes(data[self.sz_off:2 * self.sz_off], "little")
                links.update(self._symbol_table(btree, heap))
            elif mtype == 0x0006:
                name, target = _parse_link(data, self.sz_off)
                if target is not None:
                    links[name] = target
            elif mtype == 0x0002:
                # link info: a fractal-heap address means dense storage (not used by scene files)
                fh = int.from_bytes(data[2 + (8 if data[1] & 1 else 0):][:self.sz_off], "little")
                if fh != UNDEF:
                    raise H5FormatError("dense link storage (fractal heap) is not supported")
        return links

    def _heap_data(self, heap: int) -> bytes:
        p = self.base + heap
        if self._buf[p:p + 4] != b"HEAP":
            raise H5FormatError("bad local heap signature")
        size = self._uint(p + 8, self.sz_len)
        daddr = self._uint(p + 8 + 2 * self.sz_len, self.sz_off)
        return self._read(daddr, size)

    def _symbol_table(self, btree: int, heap: int) -> Dict[str, int]:
        names = self._heap_data(heap)
        out: Dict[str, int] = {}
        for snod in self._btree_children(btree, 0):
            p = self.base + snod
            if self._buf[p:p + 4] != b"SNOD":
                raise H5FormatError("bad symbol table node signature")
            n = self._uint(p + 6, 2)
            q = p + 8
            ent = 2 * self.sz_off + 24
            for i in range(n):
                e = q + i * ent
                noff = self._uint(e, self.sz_off)
                oaddr = self._uint(e + self.sz_off, self.sz_off)
                if self._uint(e + 2 * self.sz_off, 4) == 2:
                    continue  # soft link (cache type 2): not followed
                name = names[noff:names.index(b"\0", noff)].decode()
                out[name] = oaddr
        return out

    def _btree_children(self, addr: int, ntype: int) -> List[int]:
        p = self.base + addr
        b = self._buf
        if b[p:p + 4] != b"TREE" or b[p + 4] != ntype:
            raise H5FormatError("bad v1 B-tree node")
        level, used = b[p + 5], self._uint(p + 6, 2)
        q = p + 8 + 2 * self.sz_off
        ksz = self.sz_len
        kids = []
        for i in range(used):
            kids.append(self._uint(q + ksz + i * (ksz + self.sz_off), self.sz_off))
        if level == 0:
            return kids
        out = []
        for k in kids:
            out.extend(self._btree_children(k, ntype))
        return out

    def _chunk_entries(self, addr: int, rank: int):
        p = self.base + addr
        b = self._buf
        if b[p:p + 4] != b"TREE" or b[p + 4] != 1:
            raise H5FormatError("bad chunk B-tree node")
        level, used = b[p + 5], self._uint(p + 6, 2)
        ksz = 8 + 8 * (rank + 1)
        q = p + 8 + 2 * self.sz_off
        for i in range(used):
            k = q + i * (ksz + self.sz_off)
            size, fmask = self._uint(k, 4), self._uint(k + 4, 4)
            offs = [self._uint(k + 8 + 8 * d, 8) for d in range(rank)]
            child = self._uint(k + ksz, self.sz_off)
            if level == 0:
                yield size, fmask, offs, child
            else:
                yield from self._chunk_entries(child, rank)


def _parse_link(data: bytes, sz_off: int):
    flags = data[1]
    q = 2
    ltype = 0
    if flags & 0x08:
        ltype = data[q]
        q += 1
    if flags & 0x04:
        q += 8
    if flags & 0x10:
        q += 1
    nl = 1 << (flags & 3)
    n = int.from_bytes(data[q:q + nl], "little")
    q += nl
    name = data[q:q + n].decode()
    q += n
    if ltype != 0:
        return name, None  # soft / external links are not followed
    return name, int.from_bytes(data[q:q + sz_off], "little")


def _parse_dataspace(data: bytes, sz_len: int) -> Tuple[int, ...]:
    ver, rank = data[0], data[1]
    if ver == 1:
        p = 8
    elif ver == 2:
        if data[3] == 0:
            return ()  # scalar
        p = 4
    else:
        raise H5FormatError(f"unsupported dataspace version {ver}")
    return tuple(int.from_bytes(data[p + i * sz_len:p + (i + 1) * sz_len], "little") for i in range(rank))


def _parse_datatype(data: bytes) -> np.dtype:
    cls = data[0] & 0x0F
    bits = data[1]
    size = int.from_bytes(data[4:8], "little")
    order = ">" if bits & 1 else "<"
    if cls == 0:
        signed = bool(bits & 0x08)
        return np.dtype(f"{order}{'i' if signed else 'u'}{size}")
    if cls == 1:
        if size not in (2, 4, 8):
            raise H5FormatError(f"unsupported float size {size}")
        return np.dtype(f"{order}f{size}")
    raise H5FormatError(f"unsupported datatype class {cls}")


def _parse_layout(data: bytes, sz_off: int, sz_len: int):
    ver = data[0]
    if ver == 3:
        cls = data[1]
        if cls == 0:
            n = int.from_bytes(data[2:4], "little")
            return ("compact", data[4:4 + n])
        if cls == 1:
            return ("contiguous", int.from_bytes(data[2:2 + sz_off], "little"),
                    int.from_bytes(data[2 + sz_off:2 + sz_off + sz_len], "little"))
        if cls == 2:
            nd = data[2]
            addr = int.from_bytes(data[3:3 + sz_off], "little")
            dims = [int.from_bytes(data[3 + sz_off + 4 * i:7 + sz_off + 4 * i], "little") for i in range(nd)]
            return ("chunked", addr, dims)
    elif ver in (1, 2):
        nd, cls = data[1], data[2]
        p = 8
        addr = UNDEF
        if cls != 0:
            addr = int.from_bytes(data[p:p + sz_off], "little")
            p += sz_off
        dims = [int.from_bytes(data[p + 4 * i:p + 4 * i + 4], "little") for i in range(nd)]
        p += 4 * nd
        if cls == 0:
            n = int.from_bytes(data[p:p + 4], "little")
            return ("compact", data[p + 4:p + 4 + n])
        if cls == 1:
            return ("contiguous", addr, int(np.prod(dims)))
        return ("chunked", addr, dims)
    raise H5FormatError(f"unsupported layout message version {ver}")


def _parse_filters(data: bytes):
    ver, n = data[0], data[1]
    out = []
    p = 8 if ver == 1 else 2
    for _ in range(n):
        fid = int.from_bytes(data[p:p + 2], "little")
        if ver == 1 or fid >= 256:
            nlen = int.from_bytes(data[p + 2:p + 4], "little")
            p += 4
        else:
            nlen = 0
            p += 2
        nvals = int.from_bytes(data[p + 2:p + 4], "little")
        p += 4
        if ver == 1:
            nlen = (nlen + 7) // 8 * 8
        p += nlen
        vals = tuple(int.from_bytes(data[p + 4 * i:p + 4 * i + 4], "little") for i in range(nvals))
        p += 4 * nvals
        if ver == 1 and nvals % 2:
            p += 4
        out.append((fid, vals))
    return out


# ----------------------------------------------------------------------------------------- writer
def write_datasets(path: str, arrays: Dict[str, np.ndarray], compression_level: Optional[int] = 9,
                   max_chunk_bytes: int = 1 << 20) -> None:
    """Write numeric arrays as root-group datasets (the layout h5py gives `create_dataset(...,
    compression="gzip")`: superblock v0, v1 object headers, chunked + deflate)."""
    w = _Writer()
    names = sorted(arrays)
    heap_data = bytearray(b"\0" * 8)  # offset 0 = empty name (the root)
    name_off = {}
    for n in names:
        name_off[n] = len(heap_data)
        heap_data += n.encode() + b"\0"
        heap_data += b"\0" * ((-len(heap_data)) % 8)
    obj_addr = {n: w.dataset(np.ascontiguousarray(arrays[n]), compression_level, max_chunk_bytes) for n in names}
    # symbol table node (all entries in one leaf; HDF5 keeps them sorted by name)
    snod = bytearray(b"SNOD" + bytes([1, 0]) + struct.pack("<H", len(names)))
    for n in names:
        snod += struct.pack("<QQII", name_off[n], obj_addr[n], 0, 0) + b"\0" * 16
    if len(names) > 8:
        raise H5FormatError("write_datasets: at most 8 datasets (one symbol-table leaf)")
    snod += b"\0" * ((8 - len(names)) * 40)  # leaf capacity 2K = 8 entries (group leaf K = 4)
    snod_addr = w.put(bytes(snod))
    heap_seg = w.put(bytes(heap_data))
    heap = w.put(b"HEAP" + bytes([0, 0, 0, 0]) + struct.pack("<QQQ", len(heap_data), UNDEF, heap_seg))
    # group B-tree (type 0, level 0): keys are heap offsets of the boundary names
    last = name_off[names[-1]] if names else 0
    tree = b"TREE" + bytes([0, 0]) + struct.pack("<HQQ", 1 if names else 0, UNDEF, UNDEF)
    tree += struct.pack("<QQQ", 0, snod_addr, last)
    tree += b"\0" * (24 + 33 * 8 + 32 * 8 - len(tree))  # full node: 2K+1 keys, 2K children (K = 16)
    btree = w.put(tree)
    root = w.object_header([(0x0011, struct.pack("<QQ", btree, heap))])
    w.finish(path, root, btree, heap)


class _Writer:
    def __init__(self):
        self.blobs: List[bytes] = []
        self.pos = 96  # superblock v0 (56) + root symbol-table entry (40)

    def put(self, data: bytes) -> int:
        addr = self.pos
        pad = (-len(data)) % 8
        self.blobs.append(data + b"\0" * pad)
        self.pos += len(data) + pad
        return addr

    def object_header(self, msgs: List[Tuple[int, bytes]]) -> int:
        body = bytearray()
        for mtype, data in msgs:
            data = data + b"\0" * ((-len(data)) % 8)
            body += struct.pack("<HHB3x", mtype, len(data), 1 if mtype == 0x0003 else 0) + data
        hdr = struct.pack("<BBHII", 1, 0, len(msgs), 1, len(body)) + b"\0" * 4
        return self.put(hdr + bytes(body))

    def dataset(self, a: np.ndarray, level: Optional[int], max_chunk_bytes: int) -> int:
        if a.dtype.kind not in "iuf":
            raise H5FormatError(f"unsupported dtype {a.dtype}")
        a = a.astype(a.dtype.newbyteorder("<"), copy=False)
        shape = a.shape if a.ndim else (1,)
        a = a.reshape(shape)
        rank = len(shape)
        # chunks: split the leading axis so a chunk stays under max_chunk_bytes
        row_bytes = a.itemsize * int(np.prod(shape[1:], dtype=np.int64))
        rows = max(1, min(shape[0], max_chunk_bytes // max(1, row_bytes))) if shape[0] else 1
        rows = max(rows, -(-shape[0] // 64))  # one B-tree leaf holds at most 64 chunks
        cshape = (rows,) + tuple(shape[1:])
        entries = []
        for r0 in range(0, max(shape[0], 1), rows):
            block = np.zeros(cshape, dtype=a.dtype)
            part = a[r0:r0 + rows]
            block[: part.shape[0]] = part
            raw = block.tobytes()
            if level is not None:
                raw = zlib.compress(raw, level)
            entries.append((len(raw), (r0,) + (0,) * (rank - 1), self.put(raw)))
        if len(entries) > 64:
            raise H5FormatError("too many chunks for one B-tree leaf; raise max_chunk_bytes")
        ksz = 8 + 8 * (rank + 1)
        tree = bytearray(b"TREE" + bytes([1, 0]) + struct.pack("<HQQ", len(entries), UNDEF, UNDEF))
        for size, offs, addr in entries:
            tree += struct.pack("<II", size, 0) + b"".join(struct.pack("<Q", o) for o in offs) + struct.pack("<Q", 0)
            tree += struct.pack("<Q", addr)
        # final key: one past the last chunk
        tree += struct.pack("<II", 0, 0) + struct.pack("<Q", shape[0]) + b"\0" * (8 * rank)
        tree += b"\0" * (24 + 65 * ksz + 64 * 8 - len(tree))  # full node (indexed-storage K = 32)
        btree = self.put(bytes(tree))
        # messages: dataspace v1, datatype, fill value (v2, default), layout v3 chunked, filter pipeline v1
        dspace = struct.pack("<BBBB4x", 1, rank, 1, 0) + b"".join(struct.pack("<Q", d) for d in shape)
        dspace += b"".join(struct.pack("<Q", d) for d in shape)  # max dims
        if a.dtype.kind == "f":
            size = a.itemsize
            e_bits, m_bits, bias = {2: (5, 10, 15), 4: (8, 23, 127), 8: (11, 52, 1023)}[size]
            prec = 8 * size
            dtype = struct.pack("<BBBBI", 0x11, 0x20, prec - 1, 0, size)
            dtype += struct.pack("<HHBBBBI", 0, prec, m_bits, e_bits, 0, m_bits, bias)
        else:
            size = a.itemsize
            dtype = struct.pack("<BBBBI", 0x10, 0x08 if a.dtype.kind == "i" else 0, 0, 0, size)
            dtype += struct.pack("<HH", 0, 8 * size)
        fill = struct.pack("<BBBB", 2, 2, 2, 0)
        layout = struct.pack("<BBB", 3, 2, rank + 1) + struct.pack("<Q", btree)
        layout += b"".join(struct.pack("<I", c) for c in cshape) + struct.pack("<I", a.itemsize)
        msgs = [(0x0001, dspace), (0x0003, dtype), (0x0005, fill), (0x0008, layout)]
        if level is not None:
            filt = struct.pack("<BB6x", 1, 1) + struct.pack("<HHHH", 1, 8, 0, 1) + b"deflate\0"
            filt += struct.pack("<I", level) + b"\0" * 4
            msgs.append((0x000B, filt))
        return self.object_header(msgs)

    def finish(self, path: str, root: int, btree: int, heap: int) -> None:
        eof = self.pos
        sb = SIGNATURE + bytes([0, 0, 0, 0, 0, 8, 8, 0]) + struct.pack("<HHI", 4, 16, 0)
        sb += struct.pack("<QQQQ", 0, UNDEF, eof, UNDEF)
        sb += struct.pack("<QQII", 0, root, 1, 0) + struct.pack("<QQ", btree, heap)
        assert len(sb) == 96
        tmp = path + ".tmp"
        with open(tmp, "wb") as fh:
            fh.write(sb)
            for blob in self.blobs:
                fh.write(blob)
        os.replace(tmp, path)


# ----------------------------------------------------------------------------------------- scenes
SCENE_KEYS = ("triangles", "vn", "texture", "c2w", "fov")


def write_scene(path: str, triangles, vn, texture, c2w, fov, texture_dtype=np.float16,
                compression_level: Optional[int] = 9) -> None:
    """The datasets and dtypes of `scene_processor/to_h5.py:87-92` (gzip level 9); texture_dtype=np.float32
    writes the texture as other producers may (the readers keep whatever dtype the file holds).  A lower
    compression_level only changes the file's bytes, not its data (test/bench caches use 1)."""
    write_datasets(path, {
        "triangles": np.asarray(triangles, dtype=np.float32),
        "vn": np.asarray(vn, dtype=np.float32),
        "texture": np.asarray(texture, dtype=texture_dtype),
        "c2w": np.asarray(c2w, dtype=np.float32),
        "fov": np.asarray(fov, dtype=np.float32),
    }, compression_level=compression_level)


def load_single_h5_data(file_path: str):
    """`infer.py:12-30`: tensors (no batch dim) with an all-true mask."""
    import torch
    with File(file_path) as f:
        triangles = torch.from_numpy(np.array(f["triangles"]).astype(np.float32))
        texture = torch.from_numpy(np.array(f["texture"]).astype(np.float32))
        vn = torch.from_numpy(np.array(f["vn"]).astype(np.float32))
        c2w = torch.from_numpy(np.array(f["c2w"]).astype(np.float32))
        fov = torch.from_numpy(np.array(f["fov"]).astype(np.float32))
    return {"triangles": triangles, "texture": texture, "mask": torch.ones(triangles.shape[0], dtype=torch.bool),
            "c2w": c2w, "fov": fov, "vn": vn}
