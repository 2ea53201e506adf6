"""Flax-compatible msgpack (de)serialization of parameter trees.

The reference writes ``flax.serialization.msgpack_serialize(params)`` and reads
``msgpack_restore`` (/root/reference/src/main_pretrain.py:81, utils.py:151-152).  This module
re-implements that wire format with the ``msgpack`` package so checkpoints are interchangeable
with Flax without needing JAX:

* a pytree of nested ``dict``s with ``str`` keys is packed as msgpack maps;
* every array leaf is ``ExtType(1, packb((shape, dtype_name, C-order bytes)))``;
* numpy scalars are ``ExtType(3, ...)`` (same payload as arrays, restored as 0-d values);
* Python complex numbers are ``ExtType(2, packb((re, im)))``;
* arrays larger than 2**30 bytes are split into
  ``{"__msgpack_chunked_array__": True, "shape": {"0": ..}, "chunks": {"0": .., "1": ..}}``.

Decoding never executes anything from the file (msgpack only; no pickle).
"""

from __future__ import annotations

import numpy as np

try:
    import msgpack
except ImportError:  # pragma: no cover
    msgpack = None

EXT_NDARRAY = 1
EXT_COMPLEX = 2
EXT_NPSCALAR = 3
MAX_CHUNK_SIZE = 2 ** 30
CHUNK_KEY = "__msgpack_chunked_array__"


def _dtype_from_name(name):
    if isinstance(name, bytes):
        name = name.decode()
    if name == "bfloat16":
        try:
            import ml_dtypes  # noqa: F401
            return np.dtype("bfloat16")
        except Exception:
            return "bfloat16"
    return np.dtype(name)


def _arr_to_bytes(arr: np.ndarray) -> bytes:
    arr = np.asarray(arr)
    if arr.dtype.hasobject:
        raise ValueError("object arrays cannot be serialized")
    return msgpack.packb((tuple(int(s) for s in arr.shape), arr.dtype.name, arr.tobytes("C")), use_bin_type=True)


def _arr_from_bytes(data: bytes) -> np.ndarray:
    shape, dtype_name, buf = msgpack.unpackb(data, raw=True)
    dt = _dtype_from_name(dtype_name)
    if isinstance(dt, str):  # bfloat16 without ml_dtypes: widen to float32 losslessly
        raw = np.frombuffer(buf, dtype=np.uint16).astype(np.uint32) << 16
        return raw.view(np.float32).reshape(shape)
    return np.frombuffer(buf, dtype=dt).reshape(shape).copy()


def _ext_pack(x):
    if isinstance(x, np.ndarray):
        return msgpack.ExtType(EXT_NDARRAY, _arr_to_bytes(x))
    if isinstance(x, np.generic):
        return msgpack.ExtType(EXT_NPSCALAR, _arr_to_bytes(np.asarray(x)))
    if isinstance(x, complex):
        return msgpack.ExtType(EXT_COMPLEX, msgpack.packb((x.real, x.imag)))
    try:
        import torch
        if isinstance(x, torch.Tensor):
            return msgpack.ExtType(EXT_NDARRAY, _arr_to_bytes(x.detach().cpu().numpy()))
    except ImportError:  # pragma: no cover
        pass
    raise TypeError(f"cannot serialize {type(x)}")


def _ext_unpack(code, data):
    if code == EXT_NDARRAY:
        return _arr_from_bytes(data)
    if code == EXT_COMPLEX:
        re_, im = msgpack.unpackb(data)
        return complex(re_, im)
    if code == EXT_NPSCALAR:
        return _arr_from_bytes(data)[()]
    return msgpack.ExtType(code, data)


def _tuple_to_dict(t):
    return {str(i): v for i, v in enumerate(t)}


def _dict_to_tuple(d):
    return tuple(d[str(i)] for i in range(len(d)))


def _chunk(arr: np.ndarray) -> dict:
    n = max(1, MAX_CHUNK_SIZE // arr.dtype.itemsize)
    flat = arr.reshape(-1)
    chunks = [flat[i:i + n] for i in range(0, flat.size, n)]
    return {CHUNK_KEY: True, "shape": _tuple_to_dict(arr.shape), "chunks": _tuple_to_dict(chunks)}


def _prepare(tree):
    if isinstance(tree, dict):
        return {str(k): _prepare(v) for k, v in tree.items()}
    if isinstance(tree, (list, tuple)):
        return _tuple_to_dict([_prepare(v) for v in tree])
    try:
        import torch
        if isinstance(tree, torch.Tensor):
            tree = tree.detach().cpu().numpy()
    except ImportError:  # pragma: no cover
        pass
    if isinstance(tree, np.ndarray) and tree.size * tree.dtype.itemsize > MAX_CHUNK_SIZE:
        return _chunk(tree)
    return tree


def _unchunk(tree):
    if isinstance(tree, dict):
        if tree.get(CHUNK_KEY) is True:
            shape = _dict_to_tuple(tree["shape"])
            return np.concatenate(_dict_to_tuple(tree["chunks"])).reshape(shape)
        return {k: _unchunk(v) for k, v in tree.items()}
    return tree


def msgpack_serialize(tree) -> bytes:
    if msgpack is None:  # pragma: no cover
        raise RuntimeError("msgpack not installed")
    return msgpack.packb(_prepare(tree), default=_ext_pack, strict_types=True)


def msgpack_restore(data: bytes):
    if msgpack is None:  # pragma: no cover
        raise RuntimeError("msgpack not installed")
    return _unchunk(msgpack.unpackb(data, ext_hook=_ext_unpack, raw=False))


def flatten_tree(tree, prefix=()) -> dict:
    out = {}
    for k, v in tree.items():
        if isinstance(v, dict):
            out.update(flatten_tree(v, prefix + (k,)))
        else:
            out[prefix + (k,)] = v
    return out


def unflatten_tree(flat: dict) -> dict:
    tree: dict = {}
    for path, v in flat.items():
        if isinstance(path, str):
            path = tuple(path.split("/"))
        node = tree
        for k in path[:-1]:
            node = node.setdefault(k, {})
        node[path[-1]] = v
    return tree
