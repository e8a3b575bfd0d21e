"""TensorFlow checkpoint import without TensorFlow.

Reference: ``load_tf_weights_in_bert`` (bert_modeling.py:43-101) needs
TensorFlow to list and read the variables of a Google BERT checkpoint
(``bert_model.ckpt.index`` + ``bert_model.ckpt.data-00000-of-00001``) and maps
them onto the PyTorch module tree.  TensorFlow is not part of this stack, so
the V2 checkpoint ("tensor bundle") format is read directly:

* ``<prefix>.index`` is an SSTable (LevelDB table format): a 48-byte footer
  with the index-block handle, an index block of data-block handles, data
  blocks of prefix-compressed ``key -> value`` entries with a restart array,
  each block followed by a 1-byte compression type (0 none, 1 Snappy) and a
  CRC.  The value of key ``""`` is the ``BundleHeaderProto`` (shard count,
  endianness); every other key is a variable name whose value is a
  ``BundleEntryProto`` (dtype, shape, shard id, byte offset, byte size);
* ``<prefix>.data-SSSSS-of-NNNNN`` hold the raw little-endian tensor bytes.

The protobuf messages are decoded from their wire format (field numbers of
tensorflow/core/protobuf/tensor_bundle.proto and tensor_shape.proto), and
Snappy blocks are decompressed in Python.  ``write_checkpoint`` produces the
same format (uncompressed or literal-only Snappy blocks) for tests and for
exporting a model.
"""
from __future__ import annotations

import os
import re
import struct

import numpy as np

_MAGIC = 0xDB4775248B80FB57
# tensorflow/core/framework/types.proto DataType -> numpy
_DTYPES = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 5: np.int16, 6: np.int8, 9: np.int64,
           10: np.bool_, 17: np.uint16, 19: np.float16, 22: np.uint32, 23: np.uint64}
_DT_BFLOAT16 = 14
_NP_TO_DT = {np.dtype(v): k for k, v in _DTYPES.items()}


# ----------------------------------------------------------------------------- wire helpers
def _varint(buf, pos):
    shift = result = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if b < 0x80:
            return result, pos
        shift += 7


def _enc_varint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _proto_fields(buf):
    """Protobuf wire format -> {field number: [values]} (varints as int, length-delimited as bytes)."""
    out, pos = {}, 0
    while pos < len(buf):
        tag, pos = _varint(buf, pos)
        field, wt = tag >> 3, tag & 7
        if wt == 0:
            v, pos = _varint(buf, pos)
        elif wt == 1:
            v = struct.unpack_from("<Q", buf, pos)[0]
            pos += 8
        elif wt == 2:
            n, pos = _varint(buf, pos)
            v = bytes(buf[pos:pos + n])
            pos += n
        elif wt == 5:
            v = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
        else:
            raise ValueError("unsupported protobuf wire type %d" % wt)
        out.setdefault(field, []).append(v)
    return out


def _pb_varint(field, v):
    return _enc_varint(field << 3) + _enc_varint(v)


def _pb_bytes(field, b):
    return _enc_varint(field << 3 | 2) + _enc_varint(len(b)) + b


# ----------------------------------------------------------------------------- snappy
def snappy_decompress(data):
    """Raw Snappy block format (no framing): varint length, then literal / copy elements."""
    n, pos = _varint(data, 0)
    out = bytearray()
    while pos < len(data):
        tag = data[pos]
        pos += 1
        kind = tag & 3
        if kind == 0:  # literal
            ln = tag >> 2
            if ln >= 60:
                nb = ln - 59
                ln = int.from_bytes(data[pos:pos + nb], "little")
                pos += nb
            ln += 1
            out += data[pos:pos + ln]
            pos += ln
            continue
        if kind == 1:
            ln = ((tag >> 2) & 7) + 4
            off = ((tag >> 5) << 8) | data[pos]
            pos += 1
        elif kind == 2:
            ln = (tag >> 2) + 1
            off = int.from_bytes(data[pos:pos + 2], "little")
            pos += 2
        else:
            ln = (tag >> 2) + 1
            off = int.from_bytes(data[pos:pos + 4], "little")
            pos += 4
        if off == 0 or off > len(out):
            raise ValueError("corrupt snappy stream")
        for _ in range(ln):  # copies may overlap their own output
            out.append(out[-off])
    if len(out) != n:
        raise ValueError("snappy length mismatch: %d != %d" % (len(out), n))
    return bytes(out)


def snappy_compress_literal(data):
    """A valid Snappy stream made of literals only (for tests / writing)."""
    out = bytearray(_enc_varint(len(data)))
    pos = 0
    while pos < len(data):
        chunk = data[pos:pos + 65536]
        ln = len(chunk) - 1
        if ln < 60:
            out.append(ln << 2)
        else:
            nb = (ln.bit_length() + 7) // 8
            out.append((59 + nb) << 2)
            out += ln.to_bytes(nb, "little")
        out += chunk
        pos += len(chunk)
    return bytes(out)


# ----------------------------------------------------------------------------- SSTable
def _read_block(buf, offset, size):
    body = bytes(buf[offset:offset + size])
    ctype = buf[offset + size]
    if ctype == 0:
        return body
    if ctype == 1:
        return snappy_decompress(body)
    raise ValueError("unsupported SSTable block compression %d" % ctype)


def _block_entries(block):
    nrestart = struct.unpack_from("<I", block, len(block) - 4)[0]
    end = len(block) - 4 - 4 * nrestart
    pos, key = 0, b""
    while pos < end:
        shared, pos = _varint(block, pos)
        nonshared, pos = _varint(block, pos)
        vlen, pos = _varint(block, pos)
        key = key[:shared] + block[pos:pos + nonshared]
        pos += nonshared
        yield key, block[pos:pos + vlen]
        pos += vlen


def _handle(buf, pos=0):
    off, pos = _varint(buf, pos)
    size, pos = _varint(buf, pos)
    return off, size, pos


def read_table(path):
    """All ``key -> value`` entries of an SSTable file, in key order."""
    with open(path, "rb") as f:
        buf = f.read()
    if len(buf) < 48 or struct.unpack_from("<Q", buf, len(buf) - 8)[0] != _MAGIC:
        raise ValueError("%s is not an SSTable (bad footer magic)" % path)
    footer = buf[len(buf) - 48:]
    _, _, p = _handle(footer)  # metaindex handle (unused)
    ioff, isize, _ = _handle(footer, p)
    out = []
    for _, hv in _block_entries(_read_block(buf, ioff, isize)):
        doff, dsize, _ = _handle(hv)
        out.extend(_block_entries(_read_block(buf, doff, dsize)))
    return out


def _write_block(entries, compress):
    body = bytearray()
    restarts = []
    prev = b""
    for i, (k, v) in enumerate(entries):  # LevelDB layout: prefix-shared keys, a restart every 16
        shared = 0
        if i % 16 == 0:
            restarts.append(len(body))
        else:
            while shared < min(len(k), len(prev)) and k[shared] == prev[shared]:
                shared += 1
        body += _enc_varint(shared) + _enc_varint(len(k) - shared) + _enc_varint(len(v)) + k[shared:] + v
        prev = k
    if not restarts:
        restarts = [0]
    for r in restarts:
        body += struct.pack("<I", r)
    body += struct.pack("<I", len(restarts))
    body = bytes(body)
    if compress:
        return snappy_compress_literal(body), 1
    return body, 0


def write_table(path, entries, compress=False):
    entries = sorted(entries, key=lambda kv: kv[0])
    out = bytearray()

    def put(block_entries):
        data, ctype = _write_block(block_entries, compress)
        off = len(out)
        out.extend(data)
        out.append(ctype)
        out.extend(b"\0\0\0\0")  # block CRC (not verified by readers of this module)
        return off, len(data)

    doff, dsize = put(entries)
    last = entries[-1][0] if entries else b""
    moff, msize = put([])
    ioff, isize = put([(last, _enc_varint(doff) + _enc_varint(dsize))])
    footer = _enc_varint(moff) + _enc_varint(msize) + _enc_varint(ioff) + _enc_varint(isize)
    footer += b"\0" * (40 - len(footer)) + struct.pack("<Q", _MAGIC)
    out += footer
    with open(path, "wb") as f:
        f.write(out)


# ----------------------------------------------------------------------------- bundle reader
class CheckpointReader(object):
    """Variables of a TF V2 checkpoint ``prefix`` (``prefix.index`` + data shards)."""

    def __init__(self, prefix):
        if prefix.endswith(".index"):
            prefix = prefix[:-len(".index")]
        self.prefix = prefix
        self.num_shards = 1
        self.entries = {}
        for key, val in read_table(prefix + ".index"):
            f = _proto_fields(val)
            if key == b"":
                self.num_shards = f.get(1, [1])[0]
                if f.get(2, [0])[0] != 0:
                    raise ValueError("big-endian checkpoints are not supported")
                continue
            shape = []
            for sp in f.get(2, []):
                for dim in _proto_fields(sp).get(2, []):
                    shape.append(_proto_fields(dim).get(1, [0])[0])
            if f.get(7):
                raise ValueError("partitioned (sliced) variable %r is not supported" % key)
            self.entries[key.decode()] = {"dtype": f.get(1, [0])[0], "shape": tuple(shape),
                                          "shard": f.get(3, [0])[0], "offset": f.get(4, [0])[0],
                                          "size": f.get(5, [0])[0]}

    def list_variables(self):
        return [(k, list(v["shape"])) for k, v in sorted(self.entries.items())]

    def get_tensor(self, name):
        e = self.entries[name]
        path = "%s.data-%05d-of-%05d" % (self.prefix, e["shard"], self.num_shards)
        with open(path, "rb") as f:
            f.seek(e["offset"])
            raw = f.read(e["size"])
        if e["dtype"] == _DT_BFLOAT16:
            u = np.frombuffer(raw, dtype="<u2").astype(np.uint32) << 16
            return u.view(np.float32).reshape(e["shape"])
        if e["dtype"] not in _DTYPES:
            raise ValueError("variable %r has unsupported dtype %d" % (name, e["dtype"]))
        return np.frombuffer(raw, dtype=np.dtype(_DTYPES[e["dtype"]]).newbyteorder("<")).reshape(e["shape"]).copy()


def write_checkpoint(prefix, tensors, compress=False):
    """Write ``{name: ndarray}`` as a single-shard TF V2 checkpoint (``prefix.index`` + data)."""
    data = bytearray()
    entries = [(b"", _pb_varint(1, 1) + _pb_varint(2, 0) + _pb_bytes(3, _pb_varint(1, 1)))]
    for name in sorted(tensors):
        a = np.asarray(tensors[name], order="C")  # (ascontiguousarray would make scalars 1-d)
        dt = _NP_TO_DT[a.dtype]
        off = len(data)
        data += a.astype(a.dtype.newbyteorder("<")).tobytes()
        shape = b"".join(_pb_bytes(2, _pb_varint(1, d)) for d in a.shape)
        entry = _pb_varint(1, dt) + _pb_bytes(2, shape) + _pb_varint(3, 0) + _pb_varint(4, off) + \
            _pb_varint(5, a.nbytes)
        entries.append((name.encode(), entry))
    write_table(prefix + ".index", entries, compress=compress)
    with open(prefix + ".data-00000-of-00001", "wb") as f:
        f.write(data)


# ----------------------------------------------------------------------------- BERT mapping
def load_tf_weights_in_bert(model, tf_checkpoint_path, verbose=True):
    """Copy a Google BERT TF checkpoint into ``model`` with the reference's name mapping
    (bert_modeling.py:66-100): optimizer slots skipped, ``kernel`` transposed, ``gamma`` /
    ``beta`` / ``output_weights`` / ``output_bias`` renamed, ``layer_N`` indexed."""
    import torch

    reader = CheckpointReader(os.path.abspath(tf_checkpoint_path))
    for full, _shape in reader.list_variables():
        name = full.split("/")
        if any(n in ("adam_v", "adam_m", "global_step") for n in name):
            if verbose:
                print("Skipping {}".format(full))
            continue
        pointer = model
        m_name = name[-1]
        for m_name in name:
            parts = re.split(r"_(\d+)", m_name) if re.fullmatch(r"[A-Za-z]+_\d+", m_name) else [m_name]
            if parts[0] in ("kernel", "gamma", "output_weights"):
                pointer = getattr(pointer, "weight")
            elif parts[0] in ("output_bias", "beta"):
                pointer = getattr(pointer, "bias")
            else:
                pointer = getattr(pointer, parts[0])
            if len(parts) >= 2:
                pointer = pointer[int(parts[1])]
        array = reader.get_tensor(full)
        if m_name[-11:] == "_embeddings":
            pointer = getattr(pointer, "weight")
        elif m_name == "kernel":
            array = np.ascontiguousarray(np.transpose(array))
        if tuple(pointer.shape) != tuple(array.shape):
            raise ValueError("shape mismatch for {}: model {} vs checkpoint {}".format(full, tuple(pointer.shape),
                                                                                      array.shape))
        if verbose:
            print("Initialize PyTorch weight {}".format(full))
        with torch.no_grad():
            pointer.data.copy_(torch.from_numpy(array).to(pointer.dtype))
    return model
