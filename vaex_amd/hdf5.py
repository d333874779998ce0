"""Memory-mapped reader of vaex's HDF5 files, without h5py (not installed here).

vaex stores a DataFrame as contiguous HDF5 datasets -- ``/table/columns/<name>/data``
(version 2, with an optional ``mask`` dataset and an ``alias`` attribute for names HDF5
does not allow) or datasets under ``/data``, ``/columns`` or the root (version 1) -- and
maps each dataset's bytes straight into a numpy array at its file offset
(``packages/vaex-hdf5/vaex/hdf5/dataset.py:191-275,277-388``, ``dataset_mmap.py:94-110``).
This module finds those offsets by walking the file's structures itself: superblock
version 0/1, version-1 object headers with continuation blocks, symbol-table groups
(v1 B-trees, symbol-table nodes, local heaps), dataspace / datatype / layout (compact or
contiguous) messages, and attributes including variable-length strings in global heap
collections -- the subset h5py's default (earliest-format) files use, which is what vaex
writes.  Chunked or compressed datasets, newer-format groups and string columns are
reported as unsupported (the reference falls back to h5py reads there; strings are out of
this build's scope).

The mapped columns are host arrays: binning them streams them through the library's
pinned, double-buffered H2D pipeline chunk by chunk (``run_bin``), so a file larger than
HBM is processed without first loading it.
"""
import builtins
import mmap
import re
import struct

import numpy as np

SIGNATURE = b"\x89HDF\r\n\x1a\n"
UNDEF = 0xFFFFFFFFFFFFFFFF


class HDF5Error(ValueError):
    pass


class _Obj:
    """An object header: its messages as (type, payload bytes)."""

    def __init__(self, messages):
        self.messages = messages

    def first(self, mtype):
        for t, p in self.messages:
            if t == mtype:
                return p
        return None

    def all(self, mtype):
        return [p for t, p in self.messages if t == mtype]


class File:
    def __init__(self, path):
        self.path = str(path)
        self._f = builtins.open(self.path, "rb")
        self.buf = mmap.mmap(self._f.fileno(), 0, access=mmap.ACCESS_READ)
        base = -1
        for off in (0, 512, 1024, 2048, 4096, 8192):
            if self.buf[off:off + 8] == SIGNATURE:
                base = off
                break
        if base < 0:
            raise HDF5Error(f"{path}: not an HDF5 file")
        version = self.buf[base + 8]
        if version not in (0, 1):
            raise HDF5Error(f"{path}: HDF5 superblock version {version} is not supported")
        self.so, self.sl = self.buf[base + 13], self.buf[base + 14]
        if self.so != 8 or self.sl != 8:
            raise HDF5Error("only 8-byte offsets and lengths are supported")
        p = base + 24 + (4 if version == 1 else 0)
        self.base_address = self._u(p, 8)
        root_entry = p + 4 * 8
        self.root = self._entry(root_entry)

    def close(self):
        try:
            self.buf.close()
        finally:
            self._f.close()

    # ---- primitives -------------------------------------------------------------------
    def _u(self, pos, size):
        return int.from_bytes(self.buf[pos:pos + size], "little")

    def _addr(self, a):
        return a + self.base_address

    def _entry(self, pos):
        """symbol-table entry: (link name offset, object header address, cache type, scratch)"""
        name_off = self._u(pos, 8)
        header = self._u(pos + 8, 8)
        cache = self._u(pos + 16, 4)
        scratch = self.buf[pos + 24:pos + 40]
        return name_off, header, cache, scratch

    # ---- object headers -----------------------------------------------------------------
    def object(self, addr):
        a = self._addr(addr)
        version = self.buf[a]
        if version != 1:
            raise HDF5Error(f"object header version {version} is not supported (newer-format file)")
        nmsg = self._u(a + 2, 2)
        size = self._u(a + 8, 4)
        blocks = [(a + 16, size)]
        messages = []
        while blocks and len(messages) < nmsg:
            start, length = blocks.pop(0)
            pos, end = start, start + length
            while pos + 8 <= end and len(messages) < nmsg:
                mtype = self._u(pos, 2)
                msize = self._u(pos + 2, 2)
                payload = bytes(self.buf[pos + 8:pos + 8 + msize])
                pos += 8 + msize
                pos = start + ((pos - start + 7) & ~7)
                if mtype == 0x10:  # continuation
                    blocks.append((self._addr(int.from_bytes(payload[0:8], "little")),
                                   int.from_bytes(payload[8:16], "little")))
                messages.append((mtype, payload))
        return _Obj(messages)

    # ---- groups ----------------------------------------------------------------------
    def _local_heap(self, addr):
        a = self._addr(addr)
        if self.buf[a:a + 4] != b"HEAP":
            raise HDF5Error("bad local heap")
        return self._addr(self._u(a + 24, 8))

    def _heap_name(self, data_addr, off):
        end = self.buf.find(b"\x00", data_addr + off)
        return self.buf[data_addr + off:end].decode()

    def _btree_entries(self, addr, heap_data, out):
        a = self._addr(addr)
        if self.buf[a:a + 4] != b"TREE":
            raise HDF5Error("bad B-tree node")
        level = self.buf[a + 5]
        used = self._u(a + 6, 2)
        pos = a + 8 + 16  # signature, type, level, used, left, right
        children = []
        for _ in range(used):
            pos += self.sl  # key
            children.append(self._u(pos, 8))
            pos += 8
        for child in children:
            if level > 0:
                self._btree_entries(child, heap_data, out)
            else:
                self._snod(child, heap_data, out)

    def _snod(self, addr, heap_data, out):
        a = self._addr(addr)
        if self.buf[a:a + 4] != b"SNOD":
            raise HDF5Error("bad symbol table node")
        n = self._u(a + 6, 2)
        for k in range(n):
            name_off, header, _, _ = self._entry(a + 8 + 40 * k)
            out[self._heap_name(heap_data, name_off)] = header

    def members(self, obj):
        """{name: object header address} of a group (symbol-table groups only)."""
        st = obj.first(0x11)
        if st is None:
            if obj.first(0x06) is not None or obj.first(0x02) is not None:
                raise HDF5Error("newer-format (link message) groups are not supported")
            return None  # not a group
        btree, heap = int.from_bytes(st[0:8], "little"), int.from_bytes(st[8:16], "little")
        out = {}
        self._btree_entries(btree, self._local_heap(heap), out)
        return out

    # ---- datatypes, dataspaces, data -----------------------------------------------------
    def dtype(self, p):
        cls, ver = p[0] & 0x0F, p[0] >> 4
        bits = p[1] | (p[2] << 8) | (p[3] << 16)
        size = int.from_bytes(p[4:8], "little")
        order = ">" if bits & 1 else "<"
        if cls == 0:
            return np.dtype(f"{order}{'i' if bits & 8 else 'u'}{size}"), 8 + 4
        if cls == 1:
            return np.dtype(f"{order}f{size}"), 8 + 12
        if cls == 3:
            return np.dtype(f"S{size}"), 8
        if cls == 8:  # enum: h5py's bool is an int8 enum FALSE / TRUE
            base, _ = self.dtype(p[8:])
            nmem = bits & 0xFFFF
            if nmem == 2 and base.itemsize == 1:
                return np.dtype(bool), 8
            return base, 8
        if cls == 9:
            return ("vlen", bits & 0xF), 8
        raise HDF5Error(f"datatype class {cls} is not supported")

    @staticmethod
    def shape(p):
        version, ndim, flags = p[0], p[1], p[2]
        pos = 8 if version == 1 else 4
        if version == 2 and p[3] == 2:  # null dataspace
            return None
        return tuple(int.from_bytes(p[pos + 8 * k:pos + 8 * k + 8], "little") for k in range(ndim))

    def layout(self, p):
        """('contiguous', address, size) or ('compact', bytes)."""
        version = p[0]
        if version == 3:
            cls = p[1]
            if cls == 0:
                size = int.from_bytes(p[2:4], "little")
                return ("compact", p[4:4 + size])
            if cls == 1:
                return ("contiguous", int.from_bytes(p[2:10], "little"), int.from_bytes(p[10:18], "little"))
            raise HDF5Error("chunked datasets are not supported (vaex writes contiguous ones)")
        if version in (1, 2):
            ndim, cls = p[1], p[2]
            if cls == 1:
                return ("contiguous", int.from_bytes(p[8:16], "little"), None)
            raise HDF5Error("compact / chunked version-1 layouts are not supported")
        raise HDF5Error(f"layout message version {version} is not supported")

    def _global_heap_object(self, collection, index):
        a = self._addr(collection)
        if self.buf[a:a + 4] != b"GCOL":
            raise HDF5Error("bad global heap collection")
        size = self._u(a + 8, 8)
        pos, end = a + 16, a + size
        while pos + 16 <= end:
            idx = self._u(pos, 2)
            osize = self._u(pos + 8, 8)
            if idx == index:
                return bytes(self.buf[pos + 16:pos + 16 + osize])
            if idx == 0:
                break
            pos += 16 + ((osize + 7) & ~7)
        raise HDF5Error("global heap object not found")

    def attributes(self, obj):
        out = {}
        for p in obj.all(0x0C):
            version = p[0]
            if version == 1:
                nlen, tlen, slen = (int.from_bytes(p[k:k + 2], "little") for k in (2, 4, 6))
                pos = 8
                name = p[pos:pos + nlen].split(b"\x00")[0].decode()
                pos += (nlen + 7) & ~7
                tp = p[pos:pos + tlen]
                pos += (tlen + 7) & ~7
                sp = p[pos:pos + slen]
                pos += (slen + 7) & ~7
            elif version in (2, 3):
                nlen, tlen, slen = (int.from_bytes(p[k:k + 2], "little") for k in (2, 4, 6))
                pos = 8 + (1 if version == 3 else 0)
                name = p[pos:pos + nlen].split(b"\x00")[0].decode()
                pos += nlen
                tp = p[pos:pos + tlen]
                pos += tlen
                sp = p[pos:pos + slen]
                pos += slen
            else:
                continue
            try:
                dt, _ = self.dtype(tp)
                shp = self.shape(sp)
                data = p[pos:]
                count = int(np.prod(shp)) if shp else 1
                if isinstance(dt, tuple):  # variable-length string(s): (length, collection, index)
                    vals = []
                    for k in range(count):
                        q = 16 * k
                        length = int.from_bytes(data[q:q + 4], "little")
                        coll = int.from_bytes(data[q + 4:q + 12], "little")
                        index = int.from_bytes(data[q + 12:q + 16], "little")
                        vals.append(self._global_heap_object(coll, index)[:length].decode() if coll else "")
                    out[name] = vals[0] if not shp else vals
                else:
                    arr = np.frombuffer(data[:count * dt.itemsize], dt)
                    if dt.kind == "S":
                        arr = [v.split(b"\x00")[0].decode() for v in arr]
                        out[name] = arr[0] if not shp else arr
                    else:
                        out[name] = arr[0] if not shp else arr.reshape(shp)
            except HDF5Error:
                continue
        return out

    def dataset(self, obj):
        """(numpy array mapped from the file, attributes) of a dataset object header."""
        tp, sp, lp = obj.first(0x03), obj.first(0x01), obj.first(0x08)
        if tp is None or sp is None or lp is None:
            raise HDF5Error("not a dataset")
        dt, _ = self.dtype(tp)
        if isinstance(dt, tuple):
            raise HDF5Error("variable-length datasets (strings) are not supported")
        shp = self.shape(sp) or (0,)
        attrs = self.attributes(obj)
        if "dtype" in attrs and attrs["dtype"] not in ("str", "utf32"):
            dt = np.dtype(attrs["dtype"])
        lay = self.layout(lp)
        count = int(np.prod(shp))
        if lay[0] == "compact":
            arr = np.frombuffer(lay[1][:count * dt.itemsize], dt).reshape(shp)
        else:
            addr = lay[1]
            if count == 0:
                arr = np.zeros(shp, dt)
            elif addr == UNDEF:
                raise HDF5Error("dataset without storage")
            else:
                arr = np.frombuffer(self.buf, dtype=dt, count=count, offset=self._addr(addr)).reshape(shp)
        return arr, attrs


def read_columns(path):
    """{column name: array mapped from the file} in vaex's column order, plus the names of
    columns that could not be mapped (strings, chunked storage) -- dataset.py:191-388."""
    f = File(path)
    root = f.object(f.root[1])
    top = f.members(root) or {}
    columns, skipped = {}, []

    def load_group(members):
        order = []
        for name, addr in members.items():
            obj = f.object(addr)
            sub = f.members(obj)
            attrs = f.attributes(obj)
            label = attrs.get("alias", name)
            try:
                if sub is not None:  # version 2: a group per column with 'data' (+ 'mask')
                    if "data" not in sub:
                        continue
                    data, dattrs = f.dataset(f.object(sub["data"]))
                    if dattrs.get("dtype") == "str":
                        raise HDF5Error("string column")
                    if "mask" in sub:
                        mask, _ = f.dataset(f.object(sub["mask"]))
                        data = np.ma.array(data, mask=mask, shrink=False)
                else:
                    data, dattrs = f.dataset(obj)
                    label = dattrs.get("alias", label)
            except HDF5Error:
                skipped.append(label)
                continue
            if data.ndim != 1:
                skipped.append(label)
                continue
            columns[label] = data
            order.append(label)
        return order

    if "table" in top:
        table = f.object(top["table"])
        tm = f.members(table) or {}
        if "columns" in tm:
            cobj = f.object(tm["columns"])
            cm = f.members(cobj) or {}
            load_group(cm)
            order = f.attributes(cobj).get("column_order")
            if isinstance(order, str):
                wanted = [c for c in order.split(",") if c in columns]
                rest = [c for c in columns if c not in wanted]
                columns = {c: columns[c] for c in wanted + rest}
    else:
        for g in ("data", "columns"):
            if g in top:
                load_group(f.members(f.object(top[g])) or {})
        datasets = {k: v for k, v in top.items() if k not in ("data", "columns", "properties", "variables")
                    and f.members(f.object(v)) is None}
        load_group(datasets)
    return columns, skipped  # the arrays keep the file mapping alive


def open(path):
    """vaex.open for HDF5 files: a DataFrame whose columns are mapped from the file."""
    from .dataframe import DataFrame
    columns, skipped = read_columns(path)
    df = DataFrame(columns)
    df._skipped_columns = skipped
    return df


# ---------------------------------------------------------------------------- writer
# DataFrame.export_hdf5 (vaex/hdf5/export.py): the same earliest-format structures the
# reader walks -- superblock 0, version-1 object headers, one symbol-table node per group
# (the superblock's leaf K is raised so every group fits one node) -- and each column as a
# contiguous, 4 KiB-aligned dataset, so the file maps back (and DMA-streams) without copies.

_ALIGN = 4096


def _pad8(b):
    return b + b"\x00" * (-len(b) % 8)


def _msg(mtype, payload, flags=0):
    payload = _pad8(payload)
    return struct.pack("<HHB3x", mtype, len(payload), flags) + payload


def _dataspace(n):
    return struct.pack("<BBBB4xQ", 1, 1, 0, 0, n)


def _datatype(dt):
    dt = np.dtype(dt)
    if dt.kind == "b":
        dt = np.dtype("u1")
    order = 1 if dt.byteorder == ">" else 0
    if dt.kind in "iu":
        bits = order | (8 if dt.kind == "i" else 0)
        return struct.pack("<B3sI", 0x10 | 0, bits.to_bytes(3, "little"), dt.itemsize) + \
            struct.pack("<HH", 0, dt.itemsize * 8)
    if dt.kind == "f":
        if dt.itemsize == 8:
            sign, eloc, esize, msize, bias = 63, 52, 11, 52, 1023
        elif dt.itemsize == 4:
            sign, eloc, esize, msize, bias = 31, 23, 8, 23, 127
        else:
            raise HDF5Error(f"float{dt.itemsize * 8} columns are not supported")
        bits = order | (2 << 4) | (sign << 8)
        return struct.pack("<B3sI", 0x10 | 1, bits.to_bytes(3, "little"), dt.itemsize) + \
            struct.pack("<HHBBBBI", 0, dt.itemsize * 8, eloc, esize, 0, msize, bias)
    raise HDF5Error(f"columns of dtype {dt} are not supported")


def _string_attr(name, value):
    """a scalar fixed-length string attribute (attribute message version 1)"""
    data = value.encode() + b"\x00"
    nm = name.encode() + b"\x00"
    dtype = struct.pack("<B3sI", 0x10 | 3, (0).to_bytes(3, "little"), len(data))  # null-terminated ASCII
    space = struct.pack("<BBBB4x", 1, 0, 0, 0)  # scalar
    return struct.pack("<BBHHH", 1, 0, len(nm), len(dtype), len(space)) + _pad8(nm) + _pad8(dtype) + \
        _pad8(space) + data


class _Writer:
    def __init__(self):
        self.parts = []
        self.size = 0

    def alloc(self, nbytes, align=8):
        pad = -self.size % align
        if pad:
            self.parts.append(("zero", pad))
            self.size += pad
        at = self.size
        self.size += nbytes
        return at

    def put(self, data, align=8):
        at = self.alloc(len(data), align)
        self.parts.append(("bytes", data))
        return at

    def put_array(self, arr):
        at = self.alloc(arr.nbytes, _ALIGN)
        self.parts.append(("array", arr))
        return at

    def put_device(self, col):
        """an HBM column, read back in pieces when the file is written (never whole in RAM)"""
        at = self.alloc(len(col) * col.dtype.itemsize, _ALIGN)
        self.parts.append(("device", col))
        return at


def _object_header(messages):
    body = b"".join(messages)
    return struct.pack("<BBHII4x", 1, 0, len(messages), 1, len(body)) + body


def _group(w, entries, attrs=()):
    """local heap + symbol-table node + B-tree for {name: object header address};
    returns the group's object header address"""
    names = sorted(entries)
    heap = b"\x00" * 8  # offset 0: the empty string
    offs = {}
    for nm in names:
        offs[nm] = len(heap)
        heap += _pad8(nm.encode() + b"\x00")
    heap_data = w.put(heap)
    # free-list head 1 = no free block (libhdf5's H5HL_FREE_NULL)
    heap_hdr = w.put(b"HEAP" + struct.pack("<B3xQQQ", 0, len(heap), 1, heap_data))
    snod = b"SNOD" + struct.pack("<BBH", 1, 0, len(names))
    for nm in names:
        snod += struct.pack("<QQII16x", offs[nm], entries[nm], 0, 0)
    snod += b"\x00" * (40 * max(0, 2 * _LEAF_K - len(names)))
    snod_at = w.put(snod)
    last = offs[names[-1]] if names else 0
    tree = b"TREE" + struct.pack("<BBHQQ", 0, 0, 1, UNDEF, UNDEF) + struct.pack("<QQQ", 0, snod_at, last)
    tree += b"\x00" * ((2 * _INNER_K) * 16)  # room for the node's other keys / children
    tree_at = w.put(tree)
    msgs = [_msg(0x11, struct.pack("<QQ", tree_at, heap_hdr))] + [_msg(0x0C, a) for a in attrs]
    return w.put(_object_header(msgs)), tree_at, heap_hdr


_LEAF_K = 1024    # symbols per node = 2K: any DataFrame's columns fit one node
_INNER_K = 16


def export_hdf5(df, path):
    """Write df's columns (numeric, host or HBM) as vaex's HDF5 layout version 2:
    /table/columns/<name>/data contiguous datasets + column_order / alias attributes."""
    from .device import DeviceArray
    w = _Writer()
    w.put(b"\x00" * 96)  # superblock (filled in at the end)
    col_entries, order = {}, []
    for name in df.get_column_names():
        col = df.columns.get(name)
        if col is None:
            col = df.evaluate(name)
        if isinstance(col, DeviceArray) and np.dtype(col.dtype).kind in "iuf":
            store = col
            data_at = w.put_device(col)
            col = np.empty(0, col.dtype)  # dtype / kind for the header below
            nbytes, length = len(store) * store.dtype.itemsize, len(store)
        else:
            if isinstance(col, DeviceArray):
                col = col.to_numpy()
            col = np.asarray(col)
            if col.ndim != 1 or col.dtype.kind not in "biuf":
                raise HDF5Error(f"column {name!r} of dtype {col.dtype} cannot be exported")
            store = col.view(np.uint8) if col.dtype.kind == "b" else col
            data_at = w.put_array(np.ascontiguousarray(store))
            nbytes, length = store.nbytes, len(col)
        dmsgs = [_msg(0x01, _dataspace(length)), _msg(0x03, _datatype(col.dtype), flags=1),
                 _msg(0x05, struct.pack("<BBBB", 2, 2, 0, 0), flags=1),
                 _msg(0x08, struct.pack("<BBQQ", 3, 1, data_at, nbytes))]
        if col.dtype.kind == "b":
            dmsgs.append(_msg(0x0C, _string_attr("dtype", "bool")))
        data_hdr = w.put(_object_header(dmsgs))
        safe = re.sub(r"[^A-Za-z0-9_]", "_", name)
        while safe in col_entries:
            safe += "_"
        attrs = [_string_attr("alias", name)] if safe != name else []
        col_entries[safe] = _group(w, {"data": data_hdr}, attrs)[0]
        order.append(name)
    columns_hdr = _group(w, col_entries, [_string_attr("column_order", ",".join(order))])[0]
    table_hdr = _group(w, {"columns": columns_hdr})[0]
    root_hdr, root_tree, root_heap = _group(w, {"table": table_hdr})
    sb = b"\x89HDF\r\n\x1a\n" + struct.pack("<BBBBBBBBHHI", 0, 0, 0, 0, 0, 8, 8, 0, _LEAF_K, _INNER_K, 0)
    sb += struct.pack("<QQQQ", 0, UNDEF, w.size, UNDEF)
    sb += struct.pack("<QQII", 0, root_hdr, 1, 0) + struct.pack("<QQ", root_tree, root_heap)
    assert len(sb) == 96
    with builtins.open(path, "wb") as f:
        f.write(sb)
        first = True
        for kind, item in w.parts:
            if first:  # the placeholder superblock
                first = False
                continue
            if kind == "zero":
                f.write(b"\x00" * item)
            elif kind == "bytes":
                f.write(item)
            elif kind == "device":
                step = max(1, (256 << 20) // item.dtype.itemsize)
                for i in range(0, len(item), step):
                    item[i:i + step].to_numpy().tofile(f)
            else:
                item.tofile(f)
        f.truncate(w.size)
