"""Minimal HDF5 reader/writer (pure numpy) for Keras model files.

The reference saves and loads its network as a Keras HDF5 file
(``ModelCheckpoint('saved7-model-{epoch:02d}-{val_acc:.2f}.hdf5')``,
/root/reference/main.py:124; ``load_model('saved7-model-218-0.73.hdf5')``,
/root/reference/predict.py:24).  Keras writes those files through h5py with
the library defaults, i.e. the "earliest" file format: superblock v0, version-1
object headers, symbol-table groups (v1 B-tree + local heap), contiguous
datasets and fixed-length string attributes.  h5py is not part of this image,
so this module implements that subset of the HDF5 1.10 file format directly:

reader  superblock v0/v1 and v2/v3; object headers v1 and v2 (+ continuation
        blocks); groups as symbol tables (v1 B-tree, SNOD, local heap) or
        compact link messages; dataspaces v1/v2; fixed-point, IEEE float,
        fixed-length string and variable-length string (global heap) types;
        attribute messages v1-v3; data layout v3 (compact, contiguous, chunked
        over a v1 B-tree with the deflate and shuffle filters) and v4
        (compact, contiguous).
writer  superblock v0, v1 object headers, symbol-table groups, contiguous
        little-endian datasets, fixed-length string / numeric attributes --
        the layout h5py produces for a Keras ``model.save``.

Unsupported structures (dense link/attribute storage in fractal heaps, other
filters, virtual or external layouts) raise ``NotImplementedError``.  The
reader is pinned against files written by the real HDF5 C library
(tests/test_hdf5.py) and the writer's files are read back by it.
"""
from __future__ import annotations

import struct
import zlib

import numpy as np

SIGNATURE = b"\x89HDF\r\n\x1a\n"
UNDEF = 0xFFFFFFFFFFFFFFFF


class HDF5Error(ValueError):
    pass


def is_hdf5(path) -> bool:
    try:
        with open(path, "rb") as f:
            return f.read(8) == SIGNATURE
    except OSError:
        return False


def _pad8(n):
    return (n + 7) & ~7


# =============================================================================
# reader
# =============================================================================
class _Buf:
    def __init__(self, data):
        self.d = data

    def u(self, off, n):
        return int.from_bytes(self.d[off:off + n], "little")

    def bytes(self, off, n):
        if off + n > len(self.d):
            raise HDF5Error(f"read past end of file at {off:#x}+{n}")
        return bytes(self.d[off:off + n])


class Datatype:
    """Parsed datatype message: kind in {'int', 'uint', 'float', 'str', 'vlen_str'}."""

    def __init__(self, kind, size, order="<", charset=0, base=None):
        self.kind, self.size, self.order, self.charset, self.base = kind, size, order, charset, base

    def numpy(self):
        if self.kind == "float":
            return np.dtype(f"{self.order}f{self.size}")
        if self.kind == "int":
            return np.dtype(f"{self.order}i{self.size}")
        if self.kind == "uint":
            return np.dtype(f"{self.order}u{self.size}")
        if self.kind == "str":
            return np.dtype(f"S{self.size}")
        raise HDF5Error(f"no numpy dtype for {self.kind}")


def _parse_datatype(b: _Buf, off):
    cv = b.u(off, 1)
    cls, ver = cv & 0x0F, cv >> 4
    bits = b.u(off + 1, 3)
    size = b.u(off + 4, 4)
    if cls == 0:  # fixed point
        order = ">" if bits & 1 else "<"
        return Datatype("int" if bits & 8 else "uint", size, order)
    if cls == 1:  # floating point
        order = ">" if bits & 1 else "<"
        if bits & 0x40:  # VAX order
            raise NotImplementedError("VAX-ordered floats")
        return Datatype("float", size, order)
    if cls == 3:  # fixed-length string
        return Datatype("str", size, charset=(bits >> 4) & 0xF)
    if cls == 9:  # variable length
        vtype = bits & 0xF
        base = _parse_datatype(b, off + 8)
        if vtype == 1:
            return Datatype("vlen_str", size, charset=(bits >> 8) & 0xF, base=base)
        raise NotImplementedError("variable-length sequences")
    raise NotImplementedError(f"HDF5 datatype class {cls} (version {ver})")


def _parse_dataspace(b: _Buf, off, L):
    ver = b.u(off, 1)
    rank = b.u(off + 1, 1)
    flags = b.u(off + 2, 1)
    if ver == 1:
        p = off + 8
        dims = tuple(b.u(p + i * L, L) for i in range(rank))
        return dims
    if ver == 2:
        stype = b.u(off + 3, 1)
        if stype == 2:
            return None  # null dataspace
        p = off + 4
        return tuple(b.u(p + i * L, L) for i in range(rank))
    raise NotImplementedError(f"dataspace message version {ver}")


class Node:
    """An HDF5 object (group or dataset) with its attributes."""

    def __init__(self, f, addr):
        self.file = f
        self.addr = addr
        self.attrs = {}
        self._links = None  # name -> address (groups)
        self._stab = None
        self.dtype = None
        self.shape = None
        self._layout = None
        self._filters = []
        self._msgs = f._object_messages(addr)
        for mtype, moff, msize in self._msgs:
            f._apply_message(self, mtype, moff, msize)

    @property
    def is_group(self):
        return self._stab is not None or self._links is not None

    # ---- groups --------------------------------------------------------------
    def keys(self):
        return list(self._members().keys())

    def _members(self):
        if self._links is None and self._stab is not None:
            self._links = self.file._read_symbol_table(*self._stab)
        if self._links is None:
            raise HDF5Error("not a group")
        return self._links

    def __contains__(self, name):
        try:
            self[name]
            return True
        except KeyError:
            return False

    def __getitem__(self, path):
        node = self
        for part in [p for p in path.split("/") if p]:
            members = node._members()
            if part not in members:
                raise KeyError(path)
            node = self.file._node(members[part])
        return node

    # ---- datasets ------------------------------------------------------------
    def read(self):
        if self._layout is None:
            raise HDF5Error("not a dataset")
        return self.file._read_data(self)


class File:
    """Read-only HDF5 file: ``File(path)['model_weights/conv2d_1'].attrs`` etc."""

    def __init__(self, path):
        with open(path, "rb") as fh:
            self.b = _Buf(fh.read())
        self._nodes = {}
        self._parse_superblock()
        self.root = self._node(self.root_addr)
        self.attrs = self.root.attrs

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

    def __getitem__(self, path):
        return self.root[path]

    def __contains__(self, path):
        return path in self.root

    def keys(self):
        return self.root.keys()

    def _node(self, addr):
        if addr not in self._nodes:
            self._nodes[addr] = Node(self, addr)
        return self._nodes[addr]

    # ---- superblock ------------------------------------------------------------
    def _parse_superblock(self):
        b = self.b
        base = None
        for cand in (0, 512, 1024, 2048, 4096):
            if b.bytes(cand, 8) == SIGNATURE:
                base = cand
                break
        if base is None:
            raise HDF5Error("not an HDF5 file (no signature)")
        ver = b.u(base + 8, 1)
        if ver in (0, 1):
            self.O = b.u(base + 13, 1)
            self.L = b.u(base + 14, 1)
            self.leaf_k = b.u(base + 16, 2)
            self.node_k = b.u(base + 18, 2)
            p = base + 24 + (4 if ver == 1 else 0)
            self.base = b.u(p, self.O)
            p += 4 * self.O
            # root group symbol table entry: name offset, object header address, cache...
            self.root_addr = b.u(p + self.O, self.O)
        elif ver in (2, 3):
            self.O = b.u(base + 9, 1)
            self.L = b.u(base + 10, 1)
            p = base + 12
            self.base = b.u(p, self.O)
            self.root_addr = b.u(p + 3 * self.O, self.O)
            self.leaf_k, self.node_k = 4, 16
        else:
            raise NotImplementedError(f"superblock version {ver}")
        if self.O != 8 or self.L != 8:
            raise NotImplementedError("only 8-byte offsets and lengths")

    def _a(self, rel):
        return rel + self.base

    # ---- object headers --------------------------------------------------------
    def _object_messages(self, addr):
        b = self.b
        a = self._a(addr)
        msgs = []
        if b.bytes(a, 4) == b"OHDR":
            ver = b.u(a + 4, 1)
            flags = b.u(a + 5, 1)
            p = a + 6
            if flags & 0x20:
                p += 16
            if flags & 0x10:
                p += 4
            sz = 1 << (flags & 3)
            chunk = b.u(p, sz)
            p += sz
            self._v2_messages(p, p + chunk, flags, msgs)
            return msgs
        ver = b.u(a, 1)
        if ver != 1:
            raise NotImplementedError(f"object header version {ver} at {addr:#x}")
        hsize = b.u(a + 8, 4)
        self._v1_messages(a + 16, a + 16 + hsize, msgs)
        return msgs

    def _v1_messages(self, p, end, msgs):
        b = self.b
        while p + 8 <= end:
            mtype, msize = b.u(p, 2), b.u(p + 2, 2)
            data = p + 8
            if mtype == 0x10:  # continuation
                coff, clen = b.u(data, 8), b.u(data + 8, 8)
                self._v1_messages(self._a(coff), self._a(coff) + clen, msgs)
            elif mtype != 0:
                msgs.append((mtype, data, msize))
            p = data + msize

    def _v2_messages(self, p, end, hflags, msgs):
        b = self.b
        while p + 4 <= end:
            mtype, msize, mflags = b.u(p, 1), b.u(p + 1, 2), b.u(p + 3, 1)
            data = p + 4 + (2 if hflags & 0x04 else 0)
            if data + msize > end:
                break
            if mtype == 0x10:
                coff, clen = b.u(data, 8), b.u(data + 8, 8)
                c = self._a(coff)
                if b.bytes(c, 4) != b"OCHK":
                    raise HDF5Error("bad continuation block")
                self._v2_messages(c + 4, c + clen - 4, hflags, msgs)
            elif mtype != 0:
                msgs.append((mtype, data, msize))
            p = data + msize

    def _apply_message(self, node, mtype, off, size):
        b = self.b
        if mtype == 0x01:
            node.shape = _parse_dataspace(b, off, self.L)
        elif mtype == 0x03:
            node.dtype = _parse_datatype(b, off)
        elif mtype == 0x08:
            node._layout = self._parse_layout(off)
        elif mtype == 0x0B:
            node._filters = self._parse_filters(off)
        elif mtype == 0x0C:
            name, value = self._parse_attribute(off)
            node.attrs[name] = value
        elif mtype == 0x11:
            node._stab = (b.u(off, 8), b.u(off + 8, 8))
        elif mtype == 0x06:
            name, addr = self._parse_link(off)
            if node._links is None:
                node._links = {}
            if addr is not None:
                node._links[name] = addr
        elif mtype == 0x02:  # link info: dense storage if the fractal heap address is defined
            ver, flags = b.u(off, 1), b.u(off + 1, 1)
            p = off + 2 + (8 if flags & 1 else 0)
            if b.u(p, 8) != UNDEF:
                raise NotImplementedError("dense link storage (fractal heap)")
            if node._links is None:
                node._links = {}
        elif mtype == 0x15:  # attribute info
            flags = b.u(off + 1, 1)
            p = off + 2 + (2 if flags & 1 else 0)
            if b.u(p, 8) != UNDEF:
                raise NotImplementedError("dense attribute storage (fractal heap)")

    # ---- groups ----------------------------------------------------------------
    def _read_symbol_table(self, btree, heap):
        b = self.b
        h = self._a(heap)
        if b.bytes(h, 4) != b"HEAP":
            raise HDF5Error("bad local heap")
        heap_data = self._a(b.u(h + 24, 8))
        out = {}

        def name_at(o):
            s = heap_data + o
            e = self.b.d.find(b"\0", s)
            return self.b.bytes(s, e - s).decode("utf-8")

        def walk(node):
            n = self._a(node)
            sig = b.bytes(n, 4)
            if sig == b"TREE":
                level, used = b.u(n + 5, 1), b.u(n + 6, 2)
                p = n + 24
                for i in range(used):
                    child = b.u(p + 8 + i * 16, 8)
                    walk(child)
                del level
            elif sig == b"SNOD":
                nsym = b.u(n + 6, 2)
                for i in range(nsym):
                    e = n + 8 + i * 40
                    out[name_at(b.u(e, 8))] = b.u(e + 8, 8)
            else:
                raise HDF5Error(f"bad group node at {node:#x}")

        walk(btree)
        return out

    def _parse_link(self, off):
        b = self.b
        ver, flags = b.u(off, 1), b.u(off + 1, 1)
        if ver != 1:
            raise NotImplementedError(f"link message version {ver}")
        p = off + 2
        ltype = 0
        if flags & 0x08:
            ltype = b.u(p, 1)
            p += 1
        if flags & 0x04:
            p += 8
        if flags & 0x10:
            p += 1
        ls = 1 << (flags & 3)
        nlen = b.u(p, ls)
        p += ls
        name = b.bytes(p, nlen).decode("utf-8")
        p += nlen
        if ltype == 0:
            return name, b.u(p, 8)
        return name, None  # soft / external links are not followed

    # ---- attributes ------------------------------------------------------------
    def _parse_attribute(self, off):
        b = self.b
        ver = b.u(off, 1)
        nsz, tsz, ssz = b.u(off + 2, 2), b.u(off + 4, 2), b.u(off + 6, 2)
        if ver == 1:
            p = off + 8
            name = b.bytes(p, nsz).rstrip(b"\0").decode("utf-8")
            p += _pad8(nsz)
            dt = _parse_datatype(b, p)
            p += _pad8(tsz)
            shape = _parse_dataspace(b, p, self.L)
            p += _pad8(ssz)
        elif ver in (2, 3):
            p = off + 8 + (1 if ver == 3 else 0)
            name = b.bytes(p, nsz).rstrip(b"\0").decode("utf-8")
            p += nsz
            dt = _parse_datatype(b, p)
            p += tsz
            shape = _parse_dataspace(b, p, self.L)
            p += ssz
        else:
            raise NotImplementedError(f"attribute message version {ver}")
        if shape is None:
            return name, None
        n = int(np.prod(shape)) if shape else 1
        return name, self._decode(dt, b.bytes(p, n * dt.size), shape)

    def _decode(self, dt: Datatype, raw, shape):
        if dt.kind == "vlen_str":
            n = len(raw) // 16
            vals = []
            for i in range(n):
                ln = int.from_bytes(raw[16 * i:16 * i + 4], "little")
                coll = int.from_bytes(raw[16 * i + 4:16 * i + 12], "little")
                idx = int.from_bytes(raw[16 * i + 12:16 * i + 16], "little")
                vals.append(self._global_heap_object(coll, idx)[:ln])
            arr = np.array(vals, dtype=object)
        else:
            arr = np.frombuffer(raw, dtype=dt.numpy()).copy()
        return arr.reshape(shape) if shape else arr.reshape(())

    def _global_heap_object(self, coll, idx):
        b = self.b
        c = self._a(coll)
        if b.bytes(c, 4) != b"GCOL":
            raise HDF5Error("bad global heap collection")
        size = b.u(c + 8, 8)
        p, end = c + 16, c + size
        while p + 16 <= end:
            oi, osz = b.u(p, 2), b.u(p + 8, 8)
            if oi == idx:
                return b.bytes(p + 16, osz)
            if oi == 0:
                break
            p += 16 + _pad8(osz)
        raise HDF5Error(f"global heap object {idx} not found")

    # ---- datasets --------------------------------------------------------------
    def _parse_layout(self, off):
        b = self.b
        ver = b.u(off, 1)
        if ver not in (3, 4):
            raise NotImplementedError(f"data layout message version {ver}")
        cls = b.u(off + 1, 1)
        if ver == 4 and cls == 2:
            raise NotImplementedError("version-4 chunk indexes (files written with libver='latest')")
        if cls == 0:
            n = b.u(off + 2, 2)
            return ("compact", off + 4, n)
        if cls == 1:
            return ("contiguous", b.u(off + 2, 8), b.u(off + 10, 8))
        if cls == 2:
            rank = b.u(off + 2, 1)
            addr = b.u(off + 3, 8)
            dims = tuple(b.u(off + 11 + 4 * i, 4) for i in range(rank))
            return ("chunked", addr, dims)
        raise NotImplementedError(f"data layout class {cls}")

    def _parse_filters(self, off):
        b = self.b
        ver, n = b.u(off, 1), b.u(off + 1, 1)
        p = off + (8 if ver == 1 else 2)
        out = []
        for _ in range(n):
            fid = b.u(p, 2)
            if ver == 1 or fid >= 256:
                nl = b.u(p + 2, 2)
                p += 2
            else:
                nl = 0
            nv = b.u(p + 4, 2)
            p += 6
            p += _pad8(nl) if ver == 1 else nl
            vals = [b.u(p + 4 * i, 4) for i in range(nv)]
            p += 4 * nv
            if ver == 1 and nv % 2:
                p += 4
            out.append((fid, vals))
        return out

    def _read_data(self, node):
        dt, shape = node.dtype, node.shape
        if shape is None:
            return None
        n = int(np.prod(shape)) if shape else 1
        kind = node._layout[0]
        if kind == "compact":
            raw = self.b.bytes(node._layout[1], node._layout[2])
        elif kind == "contiguous":
            addr, size = node._layout[1], node._layout[2]
            if addr == UNDEF:  # never written: fill value (zeros)
                raw = bytes(n * dt.size)
            else:
                raw = self.b.bytes(self._a(addr), n * dt.size)
        else:
            return self._read_chunked(node, n)
        return self._decode(dt, raw, shape)

    def _read_chunked(self, node, n):
        dt, shape = node.dtype, node.shape
        _, btree, cdims = node._layout
        cdims = cdims[:-1]
        rank = len(shape)
        out = np.zeros(shape, dtype=dt.numpy())
        b = self.b

        def unfilter(raw, mask):
            for i, (fid, vals) in reversed(list(enumerate(node._filters))):
                if mask & (1 << i):
                    continue
                if fid == 1:
                    raw = zlib.decompress(raw)
                elif fid == 2:
                    es = vals[0] if vals else dt.size
                    a = np.frombuffer(raw, np.uint8)
                    m = len(a) // es
                    raw = a[:m * es].reshape(es, m).T.tobytes() + a[m * es:].tobytes()
                else:
                    raise NotImplementedError(f"HDF5 filter {fid}")
            return raw

        def walk(addr):
            a = self._a(addr)
            if b.bytes(a, 4) != b"TREE":
                raise HDF5Error("bad chunk B-tree")
            level, used = b.u(a + 5, 1), b.u(a + 6, 2)
            ksz = 8 + 8 * (rank + 1)
            p = a + 24
            for i in range(used):
                k = p + i * (ksz + 8)
                csize, mask = b.u(k, 4), b.u(k + 4, 4)
                offs = [b.u(k + 8 + 8 * d, 8) for d in range(rank)]
                child = b.u(k + ksz, 8)
                if level > 0:
                    walk(child)
                    continue
                raw = unfilter(b.bytes(self._a(child), csize), mask)
                blk = np.frombuffer(raw, dtype=dt.numpy())[:int(np.prod(cdims))].reshape(cdims)
                sl = tuple(slice(o, min(o + c, s)) for o, c, s in zip(offs, cdims, shape))
                out[sl] = blk[tuple(slice(0, s.stop - s.start) for s in sl)]

        if btree != UNDEF:
            walk(btree)
        return out


# =============================================================================
# writer
# =============================================================================
class _Group:
    def __init__(self):
        self.members = {}  # name -> _Group | _Dataset
        self.attrs = {}

    def create_group(self, path):
        node = self
        for part in [p for p in path.split("/") if p]:
            if part not in node.members:
                node.members[part] = _Group()
            node = node.members[part]
            if not isinstance(node, _Group):
                raise HDF5Error(f"{path}: not a group")
        return node

    def create_dataset(self, path, data):
        parts = [p for p in path.split("/") if p]
        g = self.create_group("/".join(parts[:-1])) if len(parts) > 1 else self
        if parts[-1] in g.members:
            raise HDF5Error(f"{path} exists")
        ds = _Dataset(data)
        g.members[parts[-1]] = ds
        return ds


class _Dataset:
    def __init__(self, data):
        a = np.asarray(data)
        if a.dtype.kind not in "fiu":
            raise NotImplementedError(f"dataset dtype {a.dtype}")
        self.data = a.astype(a.dtype.newbyteorder("<"), order="C", copy=True)
        self.attrs = {}


def _dt_message(a: np.ndarray):
    """Datatype message bytes (version 1) for a numpy array's element type."""
    k, sz = a.dtype.kind, a.dtype.itemsize
    if k == "f":
        if sz == 4:
            bits, props = (0x20, 31, 0), struct.pack("<HHBBBBI", 0, 32, 23, 8, 0, 23, 127)
        elif sz == 8:
            bits, props = (0x20, 63, 0), struct.pack("<HHBBBBI", 0, 64, 52, 11, 0, 52, 1023)
        elif sz == 2:
            bits, props = (0x20, 15, 0), struct.pack("<HHBBBBI", 0, 16, 10, 5, 0, 10, 15)
        else:
            raise NotImplementedError(f"float{8 * sz}")
        return bytes([0x11]) + bytes(bits) + struct.pack("<I", sz) + props
    if k in "iu":
        bits = (0x08 if k == "i" else 0, 0, 0)
        return bytes([0x10]) + bytes(bits) + struct.pack("<I", sz) + struct.pack("<HH", 0, 8 * sz)
    if k == "S":  # fixed-length, null-padded ASCII (h5py's numpy 'S' mapping)
        return bytes([0x13, 0x01, 0, 0]) + struct.pack("<I", max(sz, 1))
    raise NotImplementedError(f"attribute dtype {a.dtype}")


def _ds_message(shape):
    """Dataspace message version 1 (rank 0 = scalar)."""
    out = struct.pack("<BBBB4x", 1, len(shape), 0, 0)
    for d in shape:
        out += struct.pack("<Q", d)
    return out


def _attr_value(v):
    if isinstance(v, str):
        v = v.encode("utf-8")
    if isinstance(v, bytes):
        return np.array(v if v else b"\0", dtype=f"S{max(len(v), 1)}")
    if isinstance(v, (list, tuple)) and v and all(isinstance(x, (bytes, str)) for x in v):
        vs = [x.encode("utf-8") if isinstance(x, str) else x for x in v]
        return np.array(vs, dtype=f"S{max(1, max(len(x) for x in vs))}")
    a = np.asarray(v)
    if a.dtype.kind == "U":
        a = np.char.encode(a, "utf-8")
    if a.dtype.kind == "b":
        a = a.astype(np.int8)
    return a


def _msg(mtype, body, flags=0):
    body = body + bytes(_pad8(len(body)) - len(body))
    return struct.pack("<HHB3x", mtype, len(body), flags) + body


def _attr_message(name, value):
    a = _attr_value(value)
    if a.nbytes > 60000:
        raise NotImplementedError(f"attribute {name!r} of {a.nbytes} bytes (compact attributes are < 64 KiB)")
    nm = name.encode("utf-8") + b"\0"
    dt = _dt_message(a)
    ds = _ds_message(a.shape)
    raw = a.astype(a.dtype.newbyteorder("<")).tobytes() if a.dtype.kind != "S" else a.tobytes()
    body = struct.pack("<BBHHH", 1, 0, len(nm), len(dt), len(ds))
    body += nm + bytes(_pad8(len(nm)) - len(nm)) + dt + bytes(_pad8(len(dt)) - len(dt))
    body += ds + bytes(_pad8(len(ds)) - len(ds)) + raw
    return _msg(0x0C, body)


class Writer:
    """Build a tree of groups/datasets/attributes in memory, then ``save(path)``."""

    LEAF_K, NODE_K = 4, 16

    def __init__(self):
        self.root = _Group()
        self.attrs = self.root.attrs

    def create_group(self, path):
        return self.root.create_group(path)

    def create_dataset(self, path, data):
        return self.root.create_dataset(path, data)

    # ---- layout ----------------------------------------------------------------
    def save(self, path):
        self.buf = bytearray(96)  # superblock
        root_hdr, btree, heap = self._write_group(self.root)
        eof = len(self.buf)
        sb = SIGNATURE + bytes([0, 0, 0, 0, 0, 8, 8, 0]) + struct.pack("<HHI", self.LEAF_K, self.NODE_K, 0)
        sb += struct.pack("<QQQQ", 0, UNDEF, eof, UNDEF)
        sb += struct.pack("<QQII", 0, root_hdr, 1, 0) + struct.pack("<QQ", btree, heap)
        assert len(sb) == 96
        self.buf[0:96] = sb
        tmp = str(path) + ".tmp"
        with open(tmp, "wb") as f:
            f.write(self.buf)
        import os
        os.replace(tmp, path)

    def _alloc(self, data, align=8):
        pad = (-len(self.buf)) % align
        self.buf += bytes(pad)
        addr = len(self.buf)
        self.buf += data
        return addr

    def _object_header(self, msgs):
        body = b"".join(msgs)
        if not body:
            body = _msg(0, b"")
        hdr = struct.pack("<BBHII", 1, 0, len(msgs) or 1, 1, len(body)) + bytes(4)
        return self._alloc(hdr + body)

    def _write_dataset(self, ds: _Dataset):
        a = ds.data
        addr = self._alloc(a.tobytes(), align=8) if a.size else UNDEF
        msgs = [_msg(0x01, _ds_message(a.shape)),
                _msg(0x03, _dt_message(a), flags=1),
                _msg(0x05, struct.pack("<BBBB", 2, 2, 2, 0), flags=1),
                _msg(0x08, struct.pack("<BBQQ", 3, 1, addr, a.nbytes))]
        msgs += [_attr_message(k, v) for k, v in ds.attrs.items()]
        return self._object_header(msgs)

    def _write_group(self, g: _Group):
        """Children first, then the local heap, SNODs, B-tree and the group's header.
        Returns (header address, B-tree address, heap address)."""
        names = sorted(g.members, key=lambda s: s.encode("utf-8"))
        entries = []  # (name, header address, cache type, btree, heap)
        for nm in names:
            m = g.members[nm]
            if isinstance(m, _Group):
                h, bt, hp = self._write_group(m)
                entries.append((nm, h, 1, bt, hp))
            else:
                entries.append((nm, self._write_dataset(m), 0, 0, 0))
        # local heap: "" at offset 0, then the names (each null-terminated, 8-aligned)
        data = bytearray(8)
        offs = {}
        for nm, *_ in entries:
            offs[nm] = len(data)
            e = nm.encode("utf-8") + b"\0"
            data += e + bytes(_pad8(len(e)) - len(e))
        data_size = len(data)
        free_off = 1  # H5HL_FREE_NULL: no free block
        seg = self._alloc(bytes(data))
        heap = self._alloc(b"HEAP" + bytes([0, 0, 0, 0]) + struct.pack("<QQQ", data_size, free_off, seg))
        # symbol table nodes of at most 2*LEAF_K entries each
        cap = 2 * self.LEAF_K
        groups = [entries[i:i + cap] for i in range(0, len(entries), cap)] or [[]]
        if len(groups) > 2 * self.NODE_K:
            raise NotImplementedError(f"group with {len(entries)} members (> {2 * self.NODE_K * cap})")
        snods = []
        for grp in groups:
            body = b"SNOD" + struct.pack("<BBH", 1, 0, len(grp))
            for nm, h, ct, bt, hp in grp:
                body += struct.pack("<QQII", offs[nm], h, ct, 0) + struct.pack("<QQ", bt, hp)
            body += bytes(8 + cap * 40 - len(body))
            snods.append((self._alloc(body), offs[grp[-1][0]] if grp else 0))
        tree = b"TREE" + struct.pack("<BBH", 0, 0, len(snods) if entries else 0) + struct.pack("<QQ", UNDEF, UNDEF)
        if entries:
            tree += struct.pack("<Q", 0)
            for addr, last in snods:
                tree += struct.pack("<QQ", addr, last)
        tree += bytes(24 + (2 * self.NODE_K + 1) * 8 + 2 * self.NODE_K * 8 - len(tree))
        btree = self._alloc(tree)
        msgs = [_msg(0x11, struct.pack("<QQ", btree, heap))]
        msgs += [_attr_message(k, v) for k, v in g.attrs.items()]
        return self._object_header(msgs), btree, heap
