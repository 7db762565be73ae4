"""Minimal HDF5 writer/reader for the Keras-0.x weight file (pure Python + numpy).

The reference's only artefact is ``ModelCheckpoint(storagePath + "models/%s.mdl",
save_best_only=True)`` (cnn.py:122), i.e. Keras-0.x ``Sequential.save_weights``: an HDF5
file whose root carries attribute ``nb_layers`` and one group ``layer_{k}`` per layer with
attribute ``nb_params`` and float32 datasets ``param_{n}``. h5py is not
installed, so this module writes that file directly, in the oldest HDF5 dialect every
HDF5 library reads (the one h5py 2.x / Keras 0.x produced by default):

* superblock version 0, 8-byte offsets and lengths;
* version-1 object headers; groups are "old-style" (symbol-table message -> v1 B-tree of
  symbol-table nodes + local heap of link names);
* version-1 attribute, dataspace and datatype messages; contiguous dataset layout (v3).

Supported value types: float16/32/64, int8..int64, uint8..uint64 arrays and scalars, and
fixed-length byte strings (Python ``str`` is stored UTF-8, null-padded). The reader
understands the same dialect plus what h5py writes into such files (object-header
continuation blocks, multi-level group B-trees, compact layout, fill-value and other
messages it can skip) — enough to load weights saved by Keras 0.x itself. Files are
validated against the HDF5 C library (``h5dump``) in tests/test_h5_cpu.py.
"""
from __future__ import annotations

import struct

import numpy as np

SIGNATURE = b"\x89HDF\r\n\x1a\n"
UNDEF = 0xFFFFFFFFFFFFFFFF
_LEAF_K = 4        # group leaf node K: a symbol-table node holds up to 2K = 8 links
_INTERNAL_K = 16   # group internal node K: a B-tree node has up to 2K = 32 children
_SNOD_SIZE = 8 + 2 * _LEAF_K * 40
_BTREE_SIZE = 24 + 2 * _INTERNAL_K * 8 + (2 * _INTERNAL_K + 1) * 8
_HEAP_FREE_NULL = 1  # end-of-free-list marker of a local heap (offsets are 8-aligned)

# object-header message types
_M_NIL, _M_DSPACE, _M_DTYPE, _M_FILL_OLD, _M_FILL, _M_LAYOUT = 0x0, 0x1, 0x3, 0x4, 0x5, 0x8
_M_ATTR, _M_CONT, _M_STAB = 0xC, 0x10, 0x11


def _pad8(n: int) -> int:
    return (n + 7) & ~7


def _padded(b: bytes) -> bytes:
    return b + b"\0" * (_pad8(len(b)) - len(b))


class Group:
    """In-memory tree node: ``attrs`` name -> value, ``children`` name -> Group | ndarray."""

    def __init__(self, attrs: dict | None = None):
        self.attrs = dict(attrs or {})
        self.children: dict = {}

    def group(self, name: str, attrs: dict | None = None) -> "Group":
        g = Group(attrs)
        self.children[name] = g
        return g

    def __getitem__(self, name):
        return self.children[name]


# ------------------------------------------------------------------------------ encode
def _dtype_msg(dt: np.dtype) -> bytes:
    dt = np.dtype(dt)
    if dt.kind == "S":
        # class 3 (string), version 1; padding 1 = null pad, charset 1 = UTF-8 (ASCII superset)
        return struct.pack("<B3sI", 0x13, bytes([0x11, 0, 0]), dt.itemsize)
    order = 0 if dt.byteorder in ("<", "=", "|") else 1
    if dt.kind in "iu":
        bits = order | (0x08 if dt.kind == "i" else 0)
        return struct.pack("<B3sIHH", 0x10, bytes([bits, 0, 0]), dt.itemsize, 0, dt.itemsize * 8)
    if dt.kind == "f":
        exp_bits, man_bits, bias = {2: (5, 10, 15), 4: (8, 23, 127), 8: (11, 52, 1023)}[dt.itemsize]
        nbits = dt.itemsize * 8
        # mantissa normalisation 2 (msb implied) in bits 4-5; sign bit position in byte 1
        return struct.pack("<B3sIHHBBBBI", 0x11, bytes([order | 0x20, nbits - 1, 0]), dt.itemsize,
                           0, nbits, man_bits, exp_bits, 0, man_bits, bias)
    raise TypeError(f"unsupported HDF5 element type {dt}")


def _dspace_msg(shape) -> bytes:
    # version 1; rank 0 = scalar
    return struct.pack("<BBBB4x", 1, len(shape), 0, 0) + b"".join(struct.pack("<Q", int(d)) for d in shape)


def _as_array(v) -> np.ndarray:
    if isinstance(v, str):
        v = v.encode("utf-8")
    if isinstance(v, bytes):
        return np.array(v, dtype=f"S{max(len(v), 1)}")
    a = np.asarray(v)
    if a.dtype.kind == "U":
        a = np.char.encode(a, "utf-8")
    if a.dtype == np.bool_:
        a = a.astype(np.int8)
    if a.dtype.kind in "iuf" and a.dtype.byteorder == ">":
        a = a.astype(a.dtype.newbyteorder("<"))
    return a


def _attr_msg(name: str, value) -> bytes:
    a = _as_array(value)
    nm = name.encode("utf-8") + b"\0"
    dt, ds = _dtype_msg(a.dtype), _dspace_msg(a.shape)
    body = struct.pack("<BBHHH", 1, 0, len(nm), len(dt), len(ds))
    body += _padded(nm) + _padded(dt) + _padded(ds) + np.ascontiguousarray(a).tobytes()
    return body


def _message(mtype: int, body: bytes, flags: int = 0) -> bytes:
    body = _padded(body)
    return struct.pack("<HHB3x", mtype, len(body), flags) + body


def _object_header(messages: list) -> bytes:
    data = b"".join(messages)
    return struct.pack("<BBHII4x", 1, 0, len(messages), 1, len(data)) + data


class _Writer:
    def __init__(self):
        self.buf = bytearray(96)  # superblock, filled last

    def alloc(self, data: bytes) -> int:
        addr = _pad8(len(self.buf))
        self.buf += b"\0" * (addr - len(self.buf))
        self.buf += data
        return addr

    def dataset(self, arr) -> int:
        a = np.asarray(_as_array(arr), order="C")  # (ascontiguousarray would make 0-d 1-d)
        raw = a.tobytes()
        addr = self.alloc(raw) if raw else UNDEF
        layout = struct.pack("<BBQQ", 3, 1, addr, len(raw))           # v3, contiguous
        fill = struct.pack("<BBBB", 2, 2, 2, 0)                         # v2, late alloc, no value
        msgs = [_message(_M_DSPACE, _dspace_msg(a.shape)), _message(_M_DTYPE, _dtype_msg(a.dtype), 1),
                _message(_M_FILL, fill, 1), _message(_M_LAYOUT, layout)]
        return self.alloc(_object_header(msgs))

    def group(self, g: Group):
        """-> (object header, B-tree, local heap) addresses."""
        names = sorted(g.children, key=lambda s: s.encode("utf-8"))
        if len(names) > 2 * _LEAF_K * 2 * _INTERNAL_K:
            raise ValueError(f"group has {len(names)} links; this writer builds one B-tree level (<= 256)")
        addrs = {}
        for n in names:
            ch = g.children[n]
            addrs[n] = self.group(ch)[0] if isinstance(ch, Group) else self.dataset(ch)
        # local heap: offset 0 holds "" (the B-tree's leftmost key), then the link names
        heap, offs = bytearray(8), {}
        for n in names:
            offs[n] = len(heap)
            heap += _padded(n.encode("utf-8") + b"\0")
        heap_data = self.alloc(bytes(heap))
        heap_addr = self.alloc(b"HEAP" + struct.pack("<B3xQQQ", 0, len(heap), _HEAP_FREE_NULL, heap_data))
        # symbol-table nodes of <= 2K sorted links; B-tree key i+1 = last name of child i
        chunks = [names[i:i + 2 * _LEAF_K] for i in range(0, len(names), 2 * _LEAF_K)]
        snods = []
        for ch in chunks:
            ent = b"".join(struct.pack("<QQII16x", offs[n], addrs[n], 0, 0) for n in ch)
            node = b"SNOD" + struct.pack("<BBH", 1, 0, len(ch)) + ent
            snods.append(self.alloc(node + b"\0" * (_SNOD_SIZE - len(node))))
        bt = b"TREE" + struct.pack("<BBHQQ", 0, 0, len(snods), UNDEF, UNDEF)
        bt += struct.pack("<Q", 0)
        for ch, a in zip(chunks, snods):
            bt += struct.pack("<QQ", a, offs[ch[-1]])
        btree = self.alloc(bt + b"\0" * (_BTREE_SIZE - len(bt)))
        msgs = [_message(_M_STAB, struct.pack("<QQ", btree, heap_addr))]
        msgs += [_message(_M_ATTR, _attr_msg(k, v)) for k, v in g.attrs.items()]
        return self.alloc(_object_header(msgs)), btree, heap_addr

    def finish(self, root: Group) -> bytes:
        oh, btree, heap = self.group(root)
        eof = _pad8(len(self.buf))
        self.buf += b"\0" * (eof - len(self.buf))
        sb = SIGNATURE + struct.pack("<BBBBBBBBHHI", 0, 0, 0, 0, 0, 8, 8, 0, _LEAF_K, _INTERNAL_K, 0)
        sb += struct.pack("<QQQQ", 0, UNDEF, eof, UNDEF)
        sb += struct.pack("<QQII", 0, oh, 1, 0) + struct.pack("<QQ", btree, heap)  # root entry, cached stab
        assert len(sb) == 96
        self.buf[:96] = sb
        return bytes(self.buf)


def dumps(root: Group) -> bytes:
    return _Writer().finish(root)


def write(path: str, root: Group) -> None:
    with open(path, "wb") as f:
        f.write(dumps(root))


# ------------------------------------------------------------------------------ decode
class _Reader:
    def __init__(self, data: bytes):
        self.d = memoryview(data)
        if bytes(self.d[:8]) != SIGNATURE:
            raise ValueError("not an HDF5 file")
        ver = self.d[8]
        if ver not in (0, 1):
            raise ValueError(f"HDF5 superblock version {ver} not supported (only 0/1)")
        if self.d[13] != 8 or self.d[14] != 8:
            raise ValueError("only 8-byte offsets/lengths are supported")
        p = 24 + (4 if ver == 1 else 0)
        self.base = struct.unpack_from("<Q", self.d, p)[0]
        self.root_oh = struct.unpack_from("<Q", self.d, p + 32 + 8)[0]

    def u(self, fmt, off):
        return struct.unpack_from(fmt, self.d, self.base + off if off != UNDEF else off)

    def messages(self, addr: int) -> list:
        a = self.base + addr
        if bytes(self.d[a:a + 4]) == b"OHDR":
            raise ValueError("version-2 object headers are not supported")
        ver, _, nmsg, _, size = struct.unpack_from("<BBHII", self.d, a)
        if ver != 1:
            raise ValueError(f"object header version {ver}")
        blocks, out = [(a + 16, size)], []
        while blocks and len(out) < nmsg:
            p, n = blocks.pop(0)
            end = p + n
            while p + 8 <= end and len(out) < nmsg:
                mt, ms, _fl = struct.unpack_from("<HHB", self.d, p)
                body = bytes(self.d[p + 8:p + 8 + ms])
                p += 8 + ms
                out.append((mt, body))
                if mt == _M_CONT:
                    off, ln = struct.unpack_from("<QQ", body)
                    blocks.append((self.base + off, ln))
        return out

    def heap_name(self, heap: int, off: int) -> str:
        h = self.base + heap
        if bytes(self.d[h:h + 4]) != b"HEAP":
            raise ValueError("bad local heap")
        data = struct.unpack_from("<Q", self.d, h + 24)[0] + self.base
        end = bytes(self.d[data + off:data + off + 4096]).index(b"\0")
        return bytes(self.d[data + off:data + off + end]).decode("utf-8")

    def links(self, btree: int, heap: int) -> list:
        a = self.base + btree
        if bytes(self.d[a:a + 4]) != b"TREE":
            raise ValueError("bad group B-tree")
        ntype, level, used = struct.unpack_from("<BBH", self.d, a + 4)
        out = []
        for i in range(used):
            child = struct.unpack_from("<Q", self.d, a + 24 + 8 + 16 * i)[0]
            if level > 0:
                out += self.links(child, heap)
                continue
            s = self.base + child
            if bytes(self.d[s:s + 4]) != b"SNOD":
                raise ValueError("bad symbol-table node")
            nsym = struct.unpack_from("<H", self.d, s + 6)[0]
            for j in range(nsym):
                name_off, oh = struct.unpack_from("<QQ", self.d, s + 8 + 40 * j)
                out.append((self.heap_name(heap, name_off), oh))
        return out

    @staticmethod
    def dtype(b: bytes):
        cv, b0, b1, _b2, size = struct.unpack_from("<BBBBI", b)
        cls, ver = cv & 0x0F, cv >> 4
        end = ">" if b0 & 1 else "<"
        if cls == 0:
            return np.dtype(f"{end}{'i' if b0 & 0x08 else 'u'}{size}")
        if cls == 1:
            return np.dtype(f"{end}f{size}")
        if cls == 3:
            return np.dtype(f"S{size}")
        return None  # compound / vlen / reference ...: not needed for weight files

    @staticmethod
    def dspace(b: bytes):
        ver, rank, flags = struct.unpack_from("<BBB", b)
        if ver == 1:
            return tuple(struct.unpack_from(f"<{rank}Q", b, 8))
        if ver == 2:
            if b[3] == 2:  # null dataspace
                return None
            return tuple(struct.unpack_from(f"<{rank}Q", b, 4))
        raise ValueError(f"dataspace version {ver}")

    def attribute(self, b: bytes):
        ver = b[0]
        nlen, tlen, slen = struct.unpack_from("<HHH", b, 2)
        if ver == 1:
            p = 8
            name = b[p:p + nlen - 1].decode("utf-8"); p += _pad8(nlen)
            tb = b[p:p + tlen]; p += _pad8(tlen)
            sb = b[p:p + slen]; p += _pad8(slen)
        elif ver in (2, 3):
            p = 8 + (1 if ver == 3 else 0)
            name = b[p:p + nlen - 1].decode("utf-8"); p += nlen
            tb = b[p:p + tlen]; p += tlen
            sb = b[p:p + slen]; p += slen
        else:
            raise ValueError(f"attribute message version {ver}")
        dt, shape = self.dtype(tb), self.dspace(sb)
        if dt is None or shape is None:
            return name, None
        n = int(np.prod(shape)) if shape else 1
        a = np.frombuffer(b[p:p + n * dt.itemsize], dtype=dt).reshape(shape)
        return name, (a[()] if shape == () else a.copy())

    def dataset(self, msgs: list):
        dt = shape = layout = None
        for mt, body in msgs:
            if mt == _M_DTYPE:
                dt = self.dtype(body)
            elif mt == _M_DSPACE:
                shape = self.dspace(body)
            elif mt == _M_LAYOUT:
                layout = body
        if dt is None:
            raise ValueError("unsupported dataset element type")
        n = int(np.prod(shape)) if shape else 1
        if layout[0] != 3:
            raise ValueError(f"layout message version {layout[0]} not supported")
        if layout[1] == 1:  # contiguous
            addr, size = struct.unpack_from("<QQ", layout, 2)
            if addr == UNDEF:
                return np.zeros(shape, dt)
            raw = bytes(self.d[self.base + addr:self.base + addr + n * dt.itemsize])
        elif layout[1] == 0:  # compact
            size = struct.unpack_from("<H", layout, 2)[0]
            raw = layout[4:4 + size]
        else:
            raise ValueError("chunked (compressed) datasets are not supported")
        return np.frombuffer(raw, dtype=dt).reshape(shape).copy()

    def node(self, addr: int):
        msgs = self.messages(addr)
        stab = [body for mt, body in msgs if mt == _M_STAB]
        attrs = dict(self.attribute(body) for mt, body in msgs if mt == _M_ATTR)
        if not stab:
            return self.dataset(msgs)
        g = Group(attrs)
        btree, heap = struct.unpack_from("<QQ", stab[0])
        for name, oh in self.links(btree, heap):
            g.children[name] = self.node(oh)
        return g


def loads(data: bytes) -> Group:
    r = _Reader(data)
    return r.node(r.root_oh)


def read(path: str) -> Group:
    with open(path, "rb") as f:
        return loads(f.read())


def is_hdf5(path: str) -> bool:
    with open(path, "rb") as f:
        return f.read(8) == SIGNATURE
