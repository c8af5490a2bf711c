"""A small HDF5 reader and writer for Keras-3 `.weights.h5` checkpoints.

h5py / libhdf5 are not importable on the MI355X hosts, and the reference stores its base policy
and per-iteration checkpoints with Keras `save_weights(...weights.h5)` (agent/finetune/
train_agent.py:127-142, loaded at model/diffusion/diffusion_vpg.py:85-97). A weights file is a
tree of groups holding small float32 datasets, so the subset of the HDF5 file format (v3.0 spec)
needed for it is implemented here from the published format:

reader   superblock v0/v1/v2/v3; object headers v1 and v2 (with continuation blocks); groups as
         symbol tables (v1 B-tree + SNOD + local heap, h5py's default) or compact link messages;
         datasets with dataspace v1/v2, fixed / floating-point little- or big-endian datatypes,
         contiguous or compact layout (v1-v4). Chunked / filtered / dense-link storage raise.
writer   superblock v0, symbol-table groups, contiguous little-endian datasets (the layout h5py
         writes for Keras by default).

The reader is pinned against files written by a real HDF5 library (tests/golden/
keras_weights_h5py.weights.h5, made by tests/golden/make_h5_fixture.py with h5py), and files from
the writer are read back by h5py where it is available (tests/test_h5_cpu.py).
"""
import struct

import numpy as np

UNDEF = 0xFFFFFFFFFFFFFFFF
SIG = b"\x89HDF\r\n\x1a\n"


class H5FormatError(ValueError):
    pass


# ------------------------------------------------------------------------------------------------
# reader
# ------------------------------------------------------------------------------------------------
class _Reader:
    def __init__(self, data):
        self.b = data
        base = data.find(SIG)
        if base < 0 or base % 512:
            raise H5FormatError("not an HDF5 file (no superblock signature)")
        self.sb = base
        v = data[base + 8]
        if v in (0, 1):
            self.O, self.L = data[base + 13], data[base + 14]
            p = base + 24 + (4 if v == 1 else 0)
            self.base_addr = self._u(p, self.O)
            p += 4 * self.O                                   # base, free-space, EOF, driver
            # root group symbol table entry: link name offset, object header address, ...
            self.root = self._u(p + self.O, self.O)
        elif v in (2, 3):
            self.O, self.L = data[base + 9], data[base + 10]
            p = base + 12
            self.base_addr = self._u(p, self.O)
            self.root = self._u(p + 3 * self.O, self.O)
        else:
            raise H5FormatError(f"superblock version {v} not supported")

    def _u(self, p, n):
        return int.from_bytes(self.b[p:p + n], "little")

    def _addr(self, a):
        return self.base_addr + a

    # ---- object headers -> list of (type, data bytes) ----
    def messages(self, addr):
        p = self._addr(addr)
        b = self.b
        msgs = []
        if b[p:p + 4] == b"OHDR":
            flags = b[p + 5]
            q = p + 6
            if flags & 0x20:
                q += 16
            if flags & 0x10:
                q += 4
            nsz = 1 << (flags & 3)
            size = self._u(q, nsz)
            q += nsz
            blocks = [(q, size)]
            while blocks:
                start, size = blocks.pop(0)
                q, end = start, start + size
                while q + 4 <= end:
                    t, sz, fl = b[q], self._u(q + 1, 2), b[q + 3]
                    q += 4 + (2 if flags & 0x04 else 0)
                    d = b[q:q + sz]
                    q += sz
                    if t == 0x10:
                        ca = int.from_bytes(d[:self.O], "little")
                        cl = int.from_bytes(d[self.O:self.O + self.L], "little")
                        cp = self._addr(ca)
                        if b[cp:cp + 4] != b"OCHK":
                            raise H5FormatError("bad continuation block")
                        blocks.append((cp + 4, cl - 8))
                    elif t != 0:
                        msgs.append((t, d))
            return msgs
        if b[p] != 1:
            raise H5FormatError(f"object header version {b[p]} at {addr:#x}")
        nmsg = self._u(p + 2, 2)
        size = self._u(p + 8, 4)
        blocks = [(p + 16, size)]
        count = 0
        while blocks and count < nmsg:
            start, size = blocks.pop(0)
            q, end = start, start + size
            while q + 8 <= end and count < nmsg:
                t, sz = self._u(q, 2), self._u(q + 2, 2)
                d = b[q + 8:q + 8 + sz]
                q += 8 + sz
                count += 1
                if t == 0x10:
                    ca = int.from_bytes(d[:self.O], "little")
                    cl = int.from_bytes(d[self.O:self.O + self.L], "little")
                    blocks.append((self._addr(ca), cl))
                elif t != 0:
                    msgs.append((t, d))
        return msgs

    # ---- groups ----
    def _heap_name(self, heap, off):
        p = self._addr(heap)
        if self.b[p:p + 4] != b"HEAP":
            raise H5FormatError("bad local heap")
        data = self._u(p + 8 + 2 * self.L, self.O)
        s = self._addr(data) + off
        e = self.b.index(b"\0", s)
        return self.b[s:e].decode("utf-8")

    def _btree_children(self, addr, heap, out):
        p = self._addr(addr)
        b = self.b
        if b[p:p + 4] != b"TREE" or b[p + 4] != 0:
            raise H5FormatError("bad group B-tree node")
        level, used = b[p + 5], self._u(p + 6, 2)
        q = p + 8 + 2 * self.O
        for i in range(used):
            q += self.L                                         # key i
            child = self._u(q, self.O)
            q += self.O
            if level > 0:
                self._btree_children(child, heap, out)
            else:
                self._snod(child, heap, out)

    def _snod(self, addr, heap, out):
        p = self._addr(addr)
        b = self.b
        if b[p:p + 4] != b"SNOD":
            raise H5FormatError("bad symbol table node")
        n = self._u(p + 6, 2)
        q = p + 8
        esz = 2 * self.O + 24
        for i in range(n):
            name = self._heap_name(heap, self._u(q, self.O))
            out.append((name, self._u(q + self.O, self.O)))
            q += esz

    def _link(self, d):
        flags = d[1]
        q = 2
        ltype = 0
        if flags & 0x08:
            ltype = d[q]
            q += 1
        if flags & 0x04:
            q += 8
        if flags & 0x10:
            q += 1
        nl = 1 << (flags & 3)
        ln = int.from_bytes(d[q:q + nl], "little")
        q += nl
        name = d[q:q + ln].decode("utf-8")
        q += ln
        if ltype != 0:
            return name, None                                    # soft / external: not followed
        return name, int.from_bytes(d[q:q + self.O], "little")

    def children(self, msgs):
        out = []
        for t, d in msgs:
            if t == 0x11:
                self._btree_children(int.from_bytes(d[:self.O], "little"),
                                     int.from_bytes(d[self.O:2 * self.O], "little"), out)
            elif t == 0x06:
                name, a = self._link(d)
                if a is not None:
                    out.append((name, a))
            elif t == 0x02:
                fh = int.from_bytes(d[2 + (8 if d[1] & 1 else 0):][:self.O], "little")
                if fh != UNDEF:
                    raise H5FormatError("dense (fractal-heap) link storage is not supported")
        return out

    # ---- datasets ----
    def dataset(self, msgs):
        shape, dtype, raw = None, None, None
        for t, d in msgs:
            if t == 0x01:
                v, rank, fl = d[0], d[1], d[2]
                p = 8 if v == 1 else 4
                if v == 2 and d[3] == 2:
                    rank = 0
                shape = tuple(int.from_bytes(d[p + i * self.L:p + (i + 1) * self.L], "little") for i in range(rank))
            elif t == 0x03:
                cls, bits, size = d[0] & 0x0F, d[1], int.from_bytes(d[4:8], "little")
                endian = ">" if bits & 1 else "<"
                if cls == 1:
                    dtype = np.dtype(f"{endian}f{size}")
                elif cls == 0:
                    dtype = np.dtype(f"{endian}{'i' if bits & 0x08 else 'u'}{size}")
                else:
                    raise H5FormatError(f"datatype class {cls} is not supported")
            elif t == 0x08:
                raw = self._layout(d)
        if shape is None or dtype is None or raw is None:
            raise H5FormatError("dataset without dataspace / datatype / layout")
        n = int(np.prod(shape)) if shape else 1
        if raw == "empty":
            return np.zeros(shape, dtype)
        return np.frombuffer(raw[:n * dtype.itemsize], dtype=dtype).reshape(shape).astype(dtype.newbyteorder("="))

    def _layout(self, d):
        v = d[0]
        if v in (3, 4):                     # v4 differs from v3 only for chunked / virtual storage
            cls = d[1]
            if cls == 0:
                sz = int.from_bytes(d[2:4], "little")
                return d[4:4 + sz]
            if cls == 1:
                a = int.from_bytes(d[2:2 + self.O], "little")
                sz = int.from_bytes(d[2 + self.O:2 + self.O + self.L], "little")
                if a == UNDEF:
                    return "empty"
                return self.b[self._addr(a):self._addr(a) + sz]
            raise H5FormatError("chunked dataset storage is not supported")
        if v in (1, 2):
            rank, cls = d[1], d[2]
            q = 8
            a = None
            if cls != 0:
                a = int.from_bytes(d[q:q + self.O], "little")
                q += self.O
            dims = [int.from_bytes(d[q + 4 * i:q + 4 * i + 4], "little") for i in range(rank)]
            q += 4 * rank
            if cls == 0:
                sz = int.from_bytes(d[q:q + 4], "little")
                return d[q + 4:q + 4 + sz]
            if cls == 1:
                n = int(np.prod(dims)) if dims else 0
                return "empty" if a == UNDEF else self.b[self._addr(a):self._addr(a) + n * 8]
            raise H5FormatError("chunked dataset storage is not supported")
        raise H5FormatError(f"layout message version {v} is not supported")

    def walk(self, addr, prefix, out, seen):
        if addr in seen:
            return
        seen.add(addr)
        msgs = self.messages(addr)
        types = {t for t, _ in msgs}
        if 0x08 in types:
            out[prefix.rstrip("/")] = self.dataset(msgs)
            return
        out.setdefault("__groups__", []).append(prefix.rstrip("/"))
        for name, a in self.children(msgs):
            self.walk(a, prefix + name + "/", out, seen)


def read_h5(path):
    """{"group/sub/dataset": ndarray} for every dataset of the file; the key "__groups__" lists
    every group path ("" is the root)."""
    with open(path, "rb") as f:
        data = f.read()
    r = _Reader(data)
    out = {}
    r.walk(r.root, "", out, set())
    return out


# ------------------------------------------------------------------------------------------------
# writer (superblock v0, symbol-table groups, contiguous datasets)
# ------------------------------------------------------------------------------------------------
_LEAF_K, _NODE_K = 4, 16          # HDF5 defaults: SNOD capacity 2*4 entries, B-tree 2*16 children


def _pad8(n):
    return (n + 7) & ~7


class _Writer:
    def __init__(self):
        self.buf = bytearray(96)   # superblock, filled last

    def alloc(self, data, align=8):
        off = _pad8(len(self.buf)) if align == 8 else len(self.buf)
        self.buf.extend(b"\0" * (off - len(self.buf)))
        self.buf.extend(data)
        return off

    @staticmethod
    def ohdr_v1(messages):
        body = bytearray()
        for t, d in messages:
            d = bytes(d) + b"\0" * (_pad8(len(d)) - len(d))
            body += struct.pack("<HHB3x", t, len(d), 0) + d
        return struct.pack("<BBHII4x", 1, 0, len(messages), 1, len(body)) + bytes(body)

    def dataset(self, arr):
        a = np.asarray(arr)
        a = np.ascontiguousarray(a) if a.ndim else a.reshape(())      # keep rank 0 (scalar dataspace)
        if a.dtype.kind == "f":
            a = a.astype(a.dtype.newbyteorder("<"))
            sz = a.dtype.itemsize
            if sz == 4:
                props = struct.pack("<HHBBBBI", 0, 32, 23, 8, 0, 23, 127)
            elif sz == 8:
                props = struct.pack("<HHBBBBI", 0, 64, 52, 11, 0, 52, 1023)
            else:
                raise H5FormatError("float16 datasets are not written")
            dt = bytes([0x11, 0x20, sz * 8 - 1, 0]) + struct.pack("<I", sz) + props
        elif a.dtype.kind in "iu":
            a = a.astype(a.dtype.newbyteorder("<"))
            sz = a.dtype.itemsize
            dt = bytes([0x10, 0x08 if a.dtype.kind == "i" else 0, 0, 0]) + struct.pack("<I", sz) + \
                struct.pack("<HH", 0, sz * 8)
        else:
            raise H5FormatError(f"dtype {a.dtype} is not written")
        raw = a.tobytes()
        addr = self.alloc(raw) if raw else UNDEF
        rank = a.ndim
        space = struct.pack("<BBBB4x", 1, rank, 0, 0) + b"".join(struct.pack("<Q", n) for n in a.shape)
        fill = struct.pack("<BBBB", 2, 1, 2, 0)           # v2: early allocation, write if set, undefined
        layout = struct.pack("<BB", 3, 1) + struct.pack("<QQ", addr, len(raw))
        return self.alloc(self.ohdr_v1([(0x01, space), (0x03, dt), (0x05, fill), (0x08, layout)]))

    def group(self, children):
        """children: sorted [(name, object header address)] -> (object header addr, btree, heap)."""
        # local heap: "" at offset 0, then every name (null-terminated, 8-byte padded)
        heap = bytearray(b"\0" * 8)
        offs = []
        for name, _ in children:
            offs.append(len(heap))
            nb = name.encode("utf-8") + b"\0"
            heap += nb + b"\0" * (_pad8(len(nb)) - len(nb))
        heap_data = self.alloc(bytes(heap))
        heap_hdr = self.alloc(b"HEAP" + struct.pack("<B3xQQQ", 0, len(heap), 1, heap_data))
        # symbol table nodes of up to 2*LEAF_K entries, in name order
        cap = 2 * _LEAF_K
        chunks = [list(range(i, min(i + cap, len(children)))) for i in range(0, len(children), cap)] or [[]]
        if len(chunks) > 2 * _NODE_K:
            raise H5FormatError("group too large for one B-tree node")
        snods = []
        for ch in chunks:
            ent = bytearray()
            for i in ch:
                ent += struct.pack("<QQII16x", offs[i], children[i][1], 0, 0)
            ent += b"\0" * ((cap - len(ch)) * 40)
            snods.append(self.alloc(b"SNOD" + struct.pack("<BBH", 1, 0, len(ch)) + bytes(ent)))
        # one level-0 B-tree node: key 0 = "", key i+1 = last name of child i
        body = bytearray(struct.pack("<Q", 0))
        for ch, sn in zip(chunks, snods):
            body += struct.pack("<Q", sn)
            body += struct.pack("<Q", offs[ch[-1]] if ch else 0)
        body += b"\0" * ((2 * _NODE_K - len(chunks)) * 16)
        btree = self.alloc(b"TREE" + struct.pack("<BBHQQ", 0, 0, len(chunks), UNDEF, UNDEF) + bytes(body))
        oh = self.alloc(self.ohdr_v1([(0x11, struct.pack("<QQ", btree, heap_hdr))]))
        return oh, btree, heap_hdr

    def finish(self, root):
        oh, btree, heap = root
        sb = SIG + struct.pack("<BBBBBBBBHHI", 0, 0, 0, 0, 0, 8, 8, 0, _LEAF_K, _NODE_K, 0)
        sb += struct.pack("<QQQQ", 0, UNDEF, len(self.buf), UNDEF)
        sb += struct.pack("<QQII", 0, oh, 1, 0) + struct.pack("<QQ", btree, heap)
        assert len(sb) == 96
        self.buf[:96] = sb
        return bytes(self.buf)


def write_h5(path, datasets, groups=()):
    """datasets: {"a/b/name": ndarray}; groups: extra (possibly empty) group paths to create."""
    tree = {}

    def node(p):
        t = tree
        for part in [x for x in p.split("/") if x]:
            t = t.setdefault(part, {})
        return t
    for g in groups:
        node(g)
    for k, v in datasets.items():
        parts = [x for x in k.split("/") if x]
        node("/".join(parts[:-1]))[parts[-1]] = np.asarray(v)
    w = _Writer()

    def emit(t):
        children = []
        for name in sorted(t):
            v = t[name]
            children.append((name, emit(v)[0] if isinstance(v, dict) else w.dataset(v)))
        return w.group(children)
    root = emit(tree)
    with open(path, "wb") as f:
        f.write(w.finish(root))
