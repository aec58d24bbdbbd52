"""Keras weight files (HDF5) without h5py.

h5py is not installed on this image, but the reference's checkpoints are Keras HDF5 files:
  * Keras 2.13 saving_lib weights-only files (``model.save_weights('x.weights.h5')``,
    train_adipose_unet_v3.py:918-922): ``/layers/<layer name>/vars/<i>`` datasets (0 = kernel HWIO,
    1 = bias), ``/vars`` for the model's own variables, ``/optimizer/vars/<i>`` when compiled;
  * legacy hdf5_format files (``*.h5`` of the v2 models loaded by load_pretrained_weights,
    train_adipose_unet_v3.py:881-916, and the fallback of full_evaluation_enhanced.py:1285-1301):
    root (or ``/model_weights``) attribute ``layer_names``, per-layer attribute ``weight_names``,
    datasets ``<layer>/<weight name>`` such as ``down1_conv1/down1_conv1/kernel:0``.

This module reads and writes the subset of the HDF5 format that the HDF5 library produces for such
files with its default (earliest-format) settings, which is what h5py uses: superblock v0, version-1
object headers (with continuation blocks), symbol-table groups (v1 B-tree + local heap + symbol
nodes), contiguous or compact little-endian integer / IEEE float datasets, fixed-length string
attributes. Pinned against files written by libhdf5 1.10 itself (tests/golden/make_h5_golden.c);
files that use newer features (v2/v3 superblocks, link messages, chunked or filtered datasets,
variable-length strings) raise H5FormatError with the feature named.
"""
from __future__ import annotations

import struct
from collections import OrderedDict

import numpy as np

SIG = b"\x89HDF\r\n\x1a\n"
UNDEF = 0xFFFFFFFFFFFFFFFF


class H5FormatError(ValueError):
    pass


# ============================================================================== reader
class _Obj:
    def __init__(self):
        self.msgs = []          # (type, bytes)

    def first(self, t):
        for mt, d in self.msgs:
            if mt == t:
                return d
        return None

    def all(self, t):
        return [d for mt, d in self.msgs if mt == t]


class H5Reader:
    """Minimal read-only HDF5 file: ``tree()`` -> nested dict of groups (OrderedDict) whose leaves are
    numpy arrays; ``attrs(path)`` -> dict of attribute values."""

    def __init__(self, path):
        with open(path, "rb") as f:
            self.b = f.read()
        if self.b[:8] != SIG:
            raise H5FormatError(f"{path}: not an HDF5 file")
        ver = self.b[8]
        if ver not in (0, 1):
            raise H5FormatError(f"{path}: superblock version {ver} (only 0/1, the HDF5 default, are supported)")
        self.so, self.sl = self.b[13], self.b[14]
        if (self.so, self.sl) != (8, 8):
            raise H5FormatError("only 8-byte offsets and lengths are supported")
        p = 24 + (4 if ver == 1 else 0)
        self.base = self._u(p, 8)
        p += 32                                    # base, free-space, EOF, driver addresses
        root_entry = p
        self.root = self._u(root_entry + 8, 8)     # object header address of the root group
        self.path = path

    def _u(self, off, n):
        return int.from_bytes(self.b[off:off + n], "little")

    # ---- object headers
    def _header(self, addr):
        b = self.b
        if b[addr:addr + 4] == b"OHDR":
            raise H5FormatError("version-2 object headers are not supported")
        if b[addr] != 1:
            raise H5FormatError(f"object header version {b[addr]} at {addr}")
        nmsg = self._u(addr + 2, 2)
        size = self._u(addr + 8, 4)
        obj = _Obj()
        blocks = [(addr + 16, size)]
        while blocks and len(obj.msgs) < nmsg:
            start, length = blocks.pop(0)
            p, end = start, start + length
            while p + 8 <= end and len(obj.msgs) < nmsg:
                mt, ms, flags = self._u(p, 2), self._u(p + 2, 2), b[p + 4]
                data = b[p + 8:p + 8 + ms]
                if flags & 0x02:
                    raise H5FormatError(f"shared header message (type {mt}) not supported")
                if mt == 0x10:                    # continuation
                    blocks.append((int.from_bytes(data[0:8], "little"), int.from_bytes(data[8:16], "little")))
                obj.msgs.append((mt, data))
                p += 8 + ms
        return obj

    # ---- groups
    def _heap(self, addr):
        if self.b[addr:addr + 4] != b"HEAP":
            raise H5FormatError(f"bad local heap signature at {addr}")
        return self._u(addr + 24, 8)               # data segment address

    def _name(self, heap_data, off):
        p = heap_data + off
        e = self.b.index(b"\0", p)
        return self.b[p:e].decode("utf-8")

    def _btree_entries(self, addr, heap_data, out):
        b = self.b
        if b[addr:addr + 4] != b"TREE":
            raise H5FormatError(f"bad B-tree signature at {addr}")
        ntype, level, used = b[addr + 4], b[addr + 5], self._u(addr + 6, 2)
        if ntype != 0:
            raise H5FormatError("expected a group B-tree")
        p = addr + 24 + 8                          # skip siblings, key 0
        for _ in range(used):
            child = self._u(p, 8)
            p += 16                                # child + next key
            if level > 0:
                self._btree_entries(child, heap_data, out)
            else:
                self._snod(child, heap_data, out)

    def _snod(self, addr, heap_data, out):
        if self.b[addr:addr + 4] != b"SNOD":
            raise H5FormatError(f"bad symbol node signature at {addr}")
        n = self._u(addr + 6, 2)
        p = addr + 8
        for _ in range(n):
            name = self._name(heap_data, self._u(p, 8))
            out.append((name, self._u(p + 8, 8)))
            p += 40

    def _children(self, obj):
        st = obj.first(0x11)
        if st is None:
            if obj.first(0x06) is not None or obj.first(0x02) is not None:
                raise H5FormatError("new-style (link message) groups are not supported")
            return None
        btree, heap = int.from_bytes(st[0:8], "little"), int.from_bytes(st[8:16], "little")
        out = []
        self._btree_entries(btree, self._heap(heap), out)
        return out

    # ---- datatypes / dataspaces / data
    @staticmethod
    def _dtype(d):
        cls, ver = d[0] & 0x0F, d[0] >> 4
        bf = d[1] | (d[2] << 8) | (d[3] << 16)
        size = int.from_bytes(d[4:8], "little")
        if bf & 1 and cls in (0, 1):
            raise H5FormatError("big-endian data not supported")
        if cls == 0:
            return np.dtype(("<i" if bf & 0x08 else "<u") + str(size))
        if cls == 1:
            if size not in (2, 4, 8):
                raise H5FormatError(f"float size {size}")
            return np.dtype("<f" + str(size))
        if cls == 3:
            return np.dtype("S" + str(size))
        raise H5FormatError(f"datatype class {cls} (version {ver}) not supported")

    @staticmethod
    def _shape(d):
        ver, rank, flags = d[0], d[1], d[2]
        if ver == 1:
            p = 8
        elif ver == 2:
            if d[3] == 2:
                return None                       # null dataspace
            p = 4
        else:
            raise H5FormatError(f"dataspace version {ver}")
        return tuple(int.from_bytes(d[p + 8 * i:p + 8 * i + 8], "little") for i in range(rank))

    def _data(self, obj):
        dt = self._dtype(obj.first(0x03))
        shape = self._shape(obj.first(0x01))
        if obj.first(0x0B) is not None:
            raise H5FormatError("filtered (compressed) datasets are not supported")
        lay = obj.first(0x08)
        if lay[0] != 3:
            raise H5FormatError(f"data layout message version {lay[0]}")
        n = int(np.prod(shape)) if shape else 1
        nbytes = n * dt.itemsize
        if lay[1] == 1:                           # contiguous
            addr = int.from_bytes(lay[2:10], "little")
            raw = b"\0" * nbytes if addr == UNDEF else self.b[addr:addr + nbytes]
        elif lay[1] == 0:                         # compact
            size = int.from_bytes(lay[2:4], "little")
            raw = lay[4:4 + size]
        else:
            raise H5FormatError("chunked datasets are not supported")
        return np.frombuffer(raw, dtype=dt, count=n).reshape(shape).copy()

    def _attrs(self, obj):
        out = OrderedDict()
        for d in obj.all(0x0C):
            ver = d[0]
            if ver != 1:
                raise H5FormatError(f"attribute message version {ver}")
            nlen, tlen, slen = (int.from_bytes(d[i:i + 2], "little") for i in (2, 4, 6))
            pad = lambda x: (x + 7) & ~7  # noqa: E731
            p = 8
            name = d[p:p + nlen].split(b"\0")[0].decode("utf-8")
            p += pad(nlen)
            dt = self._dtype(d[p:p + tlen])
            p += pad(tlen)
            shape = self._shape(d[p:p + slen])
            p += pad(slen)
            n = int(np.prod(shape)) if shape else 1
            val = np.frombuffer(d[p:p + n * dt.itemsize], dtype=dt, count=n).reshape(shape)
            out[name] = val[()] if shape == () else val.copy()
        return out

    # ---- public
    def _walk(self, addr):
        obj = self._header(addr)
        kids = self._children(obj)
        if kids is None:
            return self._data(obj)
        return OrderedDict((name, self._walk(a)) for name, a in kids)

    def tree(self):
        return self._walk(self.root)

    def attrs(self, path="/"):
        addr = self.root
        for part in [p for p in path.split("/") if p]:
            kids = dict(self._children(self._header(addr)) or [])
            if part not in kids:
                raise KeyError(path)
            addr = kids[part]
        return self._attrs(self._header(addr))


def _get(tree, path):
    node = tree
    for part in [p for p in path.split("/") if p]:
        node = node[part]
    return node


def _decode(v):
    return v.decode("utf-8") if isinstance(v, bytes) else str(v)


def read_keras_weights(path):
    """-> (format, OrderedDict layer_name -> [arrays in Keras slot order]) for a Keras 2.13
    ``.weights.h5`` (saving_lib layout, format 'keras_v3') or a legacy ``.h5`` (format 'legacy')."""
    r = H5Reader(path)
    tree = r.tree()
    if "layers" in tree and isinstance(tree["layers"], dict):
        out = OrderedDict()
        for name, g in tree["layers"].items():
            vars_ = g.get("vars") if isinstance(g, dict) else None
            if not vars_:
                continue
            out[name] = [np.asarray(vars_[k]) for k in sorted(vars_, key=int)]
        return "keras_v3", out
    base = "model_weights" if "model_weights" in tree else ""
    top = r.attrs("/" + base)
    if "layer_names" not in top:
        raise KeyError(f"{path}: neither 'layers/<name>/vars' (Keras 2.13) nor a legacy 'layer_names' attribute")
    out = OrderedDict()
    for ln in top["layer_names"]:
        name = _decode(ln)
        wn = r.attrs(f"/{base}/{name}" if base else f"/{name}").get("weight_names", [])
        if len(wn) == 0:
            continue
        g = _get(tree, f"{base}/{name}")
        out[name] = [np.asarray(_get(g, _decode(w))) for w in wn]
    return "legacy", out


# ============================================================================== writer
class _Buf:
    def __init__(self):
        self.b = bytearray()

    def alloc(self, data, align=8):
        while len(self.b) % align:
            self.b.append(0)
        at = len(self.b)
        self.b += data
        return at


def _msg(mtype, data, flags=0):
    data = bytes(data)
    data += b"\0" * ((-len(data)) % 8)
    return struct.pack("<HHB3x", mtype, len(data), flags) + data


def _header_v1(msgs):
    body = b"".join(msgs)
    return struct.pack("<BBHII", 1, 0, len(msgs), 1, len(body)) + b"\0" * 4 + body


def _dt_bytes(dt):
    dt = np.dtype(dt)
    if dt.kind == "f":
        if dt.itemsize == 4:
            props = struct.pack("<HHBBBBI", 0, 32, 23, 8, 0, 23, 127)
            bf = (0x20, 31, 0)
        elif dt.itemsize == 8:
            props = struct.pack("<HHBBBBI", 0, 64, 52, 11, 0, 52, 1023)
            bf = (0x20, 63, 0)
        else:
            raise H5FormatError(f"float{dt.itemsize * 8} not supported")
        return bytes([0x11, *bf]) + struct.pack("<I", dt.itemsize) + props
    if dt.kind in "iu":
        bf = 0x08 if dt.kind == "i" else 0
        return bytes([0x10, bf, 0, 0]) + struct.pack("<I", dt.itemsize) + struct.pack("<HH", 0, dt.itemsize * 8)
    if dt.kind == "S":
        return bytes([0x13, 0x01, 0, 0]) + struct.pack("<I", dt.itemsize)   # null-padded ASCII
    raise H5FormatError(f"dtype {dt} not supported")


def _ds_bytes(shape):
    return struct.pack("<BBBx4x", 1, len(shape), 0) + b"".join(struct.pack("<Q", d) for d in shape)


def _attr_msg(name, value):
    v = np.asarray(value)
    if v.dtype.kind == "U":
        v = np.char.encode(v, "utf-8")
    if v.dtype.kind == "S" and v.dtype.itemsize == 0:
        v = v.astype("S1")
    nm = name.encode("utf-8") + b"\0"
    dt, ds = _dt_bytes(v.dtype), _ds_bytes(v.shape)
    pad = lambda x: x + b"\0" * ((-len(x)) % 8)  # noqa: E731
    data = struct.pack("<BxHHH", 1, len(nm), len(dt), len(ds)) + pad(nm) + pad(dt) + pad(ds) + v.tobytes()
    return _msg(0x0C, data)


class H5Writer:
    """Builds an HDF5 file from a nested dict: dict = group, numpy array = dataset; ``attrs`` maps a
    group path ('/' or 'a/b') to {name: value}. Layout: superblock v0, version-1 object headers,
    symbol-table groups (leaf K 4 / internal K 16, the library defaults), contiguous datasets."""

    LEAF_K, NODE_K = 4, 16

    def __init__(self, tree, attrs=None):
        self.tree = tree
        self.attrs = {("/" + k.strip("/")) if k != "/" else "/": v for k, v in (attrs or {}).items()}
        self.buf = _Buf()

    def _dataset(self, arr):
        arr = np.ascontiguousarray(arr)
        if arr.dtype.byteorder == ">":
            arr = arr.astype(arr.dtype.newbyteorder("<"))
        addr = self.buf.alloc(arr.tobytes()) if arr.nbytes else UNDEF
        msgs = [_msg(0x01, _ds_bytes(arr.shape)), _msg(0x03, _dt_bytes(arr.dtype), flags=1),
                _msg(0x05, bytes([2, 2, 2, 0])),                       # fill value v2: undefined
                _msg(0x08, struct.pack("<BBQQ", 3, 1, addr, arr.nbytes))]
        return self.buf.alloc(_header_v1(msgs))

    def _group(self, node, path):
        kids = []
        for name in sorted(node):                  # symbol nodes hold entries in name order
            child = node[name]
            cpath = (path.rstrip("/") + "/" + name)
            kids.append((name, self._group(child, cpath) if isinstance(child, dict) else self._dataset(child)))
        # local heap: "" at 0, then the names (8-byte aligned)
        heap = bytearray(b"\0" * 8)
        offs = []
        for name, _ in kids:
            offs.append(len(heap))
            nb = name.encode("utf-8") + b"\0"
            heap += nb + b"\0" * ((-len(nb)) % 8)
        heap_data = self.buf.alloc(bytes(heap))    # no free block: free-list head = 1 (H5HL_FREE_NULL)
        heap_hdr = self.buf.alloc(b"HEAP" + struct.pack("<B3xQQQ", 0, len(heap), 1, heap_data))
        # symbol nodes of <= 2*LEAF_K entries, one B-tree leaf over them
        cap = 2 * self.LEAF_K
        chunks = [list(range(i, min(i + cap, len(kids)))) for i in range(0, len(kids), cap)] or [[]]
        if len(chunks) > 2 * self.NODE_K:
            raise H5FormatError(f"group {path}: more than {2 * self.NODE_K * cap} entries")
        snods = []
        for ch in chunks:
            ent = b"".join(struct.pack("<QQI4x16x", offs[i], kids[i][1], 0) for i in ch)
            ent += b"\0" * (40 * (cap - len(ch)))
            snods.append(self.buf.alloc(b"SNOD" + struct.pack("<BxH", 1, len(ch)) + ent))
        nk = 2 * self.NODE_K
        tree = b"TREE" + struct.pack("<BBHQQ", 0, 0, len(snods), UNDEF, UNDEF) + struct.pack("<Q", 0)
        for ch, sn in zip(chunks, snods):
            tree += struct.pack("<QQ", sn, offs[ch[-1]] if ch else 0)
        tree += b"\0" * (16 * (nk - len(snods)))
        btree = self.buf.alloc(tree)
        msgs = [_msg(0x11, struct.pack("<QQ", btree, heap_hdr))]
        for k, v in (self.attrs.get(path) or {}).items():
            msgs.append(_attr_msg(k, v))
        addr = self.buf.alloc(_header_v1(msgs))
        if path == "/":
            self.root_cache = (btree, heap_hdr)
        return addr

    def write(self, filename):
        self.buf.alloc(b"\0" * 96)                 # superblock, patched below
        root = self._group(self.tree, "/")
        eof = len(self.buf.b)
        sb = SIG + bytes([0, 0, 0, 0, 0, 8, 8, 0]) + struct.pack("<HHI", self.LEAF_K, self.NODE_K, 0)
        sb += struct.pack("<QQQQ", 0, UNDEF, eof, UNDEF)
        sb += struct.pack("<QQI4xQQ", 0, root, 1, *self.root_cache)
        assert len(sb) == 96
        self.buf.b[0:96] = sb
        with open(filename, "wb") as f:
            f.write(bytes(self.buf.b))


def write_keras_weights(path, layers, fmt="keras_v3", keras_version="2.13.1"):
    """layers: OrderedDict layer_name -> [arrays in Keras slot order]. fmt 'keras_v3' writes the Keras 2.13
    saving_lib layout (``*.weights.h5``), 'legacy' the hdf5_format layout (``*.h5``)."""
    if fmt == "keras_v3":
        tree = OrderedDict([("layers", OrderedDict()), ("vars", OrderedDict())])
        for name, arrs in layers.items():
            tree["layers"][name] = OrderedDict(
                [("vars", OrderedDict((str(i), np.asarray(a)) for i, a in enumerate(arrs)))])
        H5Writer(tree).write(path)
        return path
    if fmt != "legacy":
        raise ValueError(f"unknown weight file format {fmt!r}")
    tree, attrs = OrderedDict(), {}
    slot_names = ("kernel:0", "bias:0", "gamma:0", "beta:0", "moving_mean:0", "moving_variance:0")
    for name, arrs in layers.items():
        wn = [f"{name}/{slot_names[i] if i < len(slot_names) else f'w{i}:0'}" for i in range(len(arrs))]
        g = OrderedDict()
        for w, a in zip(wn, arrs):
            g.setdefault(name, OrderedDict())[w.split("/", 1)[1]] = np.asarray(a)
        tree[name] = g
        attrs[name] = {"weight_names": np.array([w.encode() for w in wn])}
    attrs["/"] = {"layer_names": np.array([n.encode() for n in layers]), "backend": np.bytes_(b"tensorflow"),
                  "keras_version": np.bytes_(keras_version.encode())}
    H5Writer(tree, attrs).write(path)
    return path
