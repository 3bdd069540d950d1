"""Minimal ONNX (protobuf wire format) reader for the xiaoa weights.

The reference ships the trained CNN as ``ml_models/xiaoa.onnx`` (opset 18,
exported by PyTorch 2.1; graph input ``input.1 [1,13,63]``, output ``22``).
No code in the reference loads it for inference and neither ``onnx`` nor
``onnxruntime`` is available, so this module decodes the protobuf directly:
only ``ModelProto.graph`` (field 7) -> ``GraphProto.initializer`` (5),
``input`` (11), ``output`` (12) and ``TensorProto`` {dims 1, data_type 2,
float_data 4, name 8, raw_data 9} are read.  Nothing in the file is executed.
"""
from __future__ import annotations

import struct
from typing import Dict, List, Tuple

import numpy as np

_ONNX_FLOAT = 1
_ONNX_DTYPES = {1: np.float32, 2: np.uint8, 3: np.int8, 5: np.int16, 6: np.int32, 7: np.int64,
                10: np.float16, 11: np.float64}


def _varint(buf: bytes, pos: int) -> Tuple[int, int]:
    result = 0
    shift = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7
        if shift > 70:
            raise ValueError("malformed varint")


def _fields(buf: bytes):
    """Yield (field_number, wire_type, value) over one protobuf message."""
    pos, end = 0, len(buf)
    while pos < end:
        key, pos = _varint(buf, pos)
        field, wt = key >> 3, key & 7
        if wt == 0:
            val, pos = _varint(buf, pos)
        elif wt == 1:
            val = buf[pos:pos + 8]
            pos += 8
        elif wt == 2:
            ln, pos = _varint(buf, pos)
            val = buf[pos:pos + ln]
            pos += ln
        elif wt == 5:
            val = buf[pos:pos + 4]
            pos += 4
        else:
            raise ValueError(f"unsupported wire type {wt}")
        if pos > end:
            raise ValueError("truncated protobuf message")
        yield field, wt, val


def _tensor(buf: bytes) -> Tuple[str, np.ndarray]:
    dims: List[int] = []
    dtype = _ONNX_FLOAT
    name = ""
    raw = None
    floats: List[float] = []
    for f, wt, v in _fields(buf):
        if f == 1:
            if wt == 2:  # packed
                p = 0
                while p < len(v):
                    d, p = _varint(v, p)
                    dims.append(d)
            else:
                dims.append(v)
        elif f == 2:
            dtype = v
        elif f == 4:
            if wt == 2:
                floats.extend(struct.unpack(f"<{len(v) // 4}f", v))
            else:
                floats.append(struct.unpack("<f", v)[0])
        elif f == 8:
            name = v.decode("utf-8")
        elif f == 9:
            raw = v
    if dtype not in _ONNX_DTYPES:
        raise ValueError(f"initializer {name!r}: unsupported ONNX dtype {dtype}")
    np_dtype = _ONNX_DTYPES[dtype]
    if raw is not None:
        arr = np.frombuffer(raw, dtype=np.dtype(np_dtype).newbyteorder("<")).astype(np_dtype)
    else:
        arr = np.asarray(floats, dtype=np_dtype)
    return name, arr.reshape(dims) if dims else arr


def _value_info_name(buf: bytes) -> str:
    for f, _, v in _fields(buf):
        if f == 1:
            return v.decode("utf-8")
    return ""


def read_onnx(path: str) -> Tuple[Dict[str, np.ndarray], List[str], List[str]]:
    """Return (initializers by name, graph input names, graph output names)."""
    with open(path, "rb") as fh:
        model = fh.read()
    graph = None
    for f, wt, v in _fields(model):
        if f == 7 and wt == 2:
            graph = v
    if graph is None:
        raise ValueError(f"{path}: no GraphProto in ONNX model")
    inits: Dict[str, np.ndarray] = {}
    inputs: List[str] = []
    outputs: List[str] = []
    for f, wt, v in _fields(graph):
        if f == 5:
            name, arr = _tensor(v)
            inits[name] = arr
        elif f == 11:
            inputs.append(_value_info_name(v))
        elif f == 12:
            outputs.append(_value_info_name(v))
    inputs = [n for n in inputs if n not in inits]
    return inits, inputs, outputs


def xiaoa_state_dict(inits: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
    """Map ONNX initializers to LightweightKWS state-dict keys
    (wakeModel.py:8-27).  The exporter folded the two bias-free Linear layers
    into MatMul weights stored [in, out]; transpose them back to [out, in]."""
    conv = [k for k in ("conv_layers.0.weight", "conv_layers.3.weight", "conv_layers.6.weight") if k in inits]
    mm = sorted((k for k in inits if k.startswith("onnx::MatMul_")), key=lambda s: int(s.rsplit("_", 1)[1]))
    if len(conv) != 3 or len(mm) != 2:
        raise ValueError("ONNX graph is not a bias-free LightweightKWS export "
                         f"(conv initializers {conv}, matmul initializers {mm})")
    sd = {k: np.ascontiguousarray(inits[k], np.float32) for k in conv}
    sd["classifier.0.weight"] = np.ascontiguousarray(inits[mm[0]].T, np.float32)
    sd["classifier.2.weight"] = np.ascontiguousarray(inits[mm[1]].T, np.float32)
    expect = {"conv_layers.0.weight": (32, 13, 3), "conv_layers.3.weight": (64, 32, 3),
              "conv_layers.6.weight": (128, 64, 3), "classifier.0.weight": (64, 128),
              "classifier.2.weight": (1, 64)}
    for k, shp in expect.items():
        if sd[k].shape != shp:
            raise ValueError(f"{k}: shape {sd[k].shape}, expected {shp}")
    return sd
