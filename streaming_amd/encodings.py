"""MDS column encodings: the host side of the codec registry.

Mirrors the encoding names, fixed sizes and byte formats of the reference codec registry
(``streaming/base/format/mds/encodings.py:654-683``, ``_get_coder`` at ``:697-714``). The
device decodes every column's bytes; this module supplies what is inherently host work:

* ``parse_encoding`` -- name / dtype / shape / fixed size of an encoding string (the same facts
  ``mdsx_plan_create`` derives in C++), used to shape the torch outputs;
* ``mds_encode`` / ``get_mds_encoded_size`` / ``is_mds_encoding`` -- the writer side, used by
  :class:`streaming_amd.writer.MDSWriter` (``encodings.py:742-757,776-788``);
* ``host_object_decode`` -- Python-object construction for the encodings whose decoded value
  is a Python object (``pil``, ``jpeg``, ``png``, ``list[*]``, ``jpeg_array``, ``pkl``,
  ``json``, ``str_int``/``str_float``/``str_decimal``; ``encodings.py:410-650``), applied to
  bytes the device already gathered; and the header split of dynamic ndarrays.
"""

from __future__ import annotations

import json
import pickle
from dataclasses import dataclass
from decimal import Decimal
from io import BytesIO
from typing import Any, Optional

import numpy as np

__all__ = [
    'EncodingInfo', 'parse_encoding', 'get_mds_encodings', 'is_mds_encoding',
    'is_mds_encoding_safe', 'get_mds_encoded_size', 'mds_encode', 'host_object_decode',
    'ndarray_dyn_decode', 'VALUE_DTYPES', 'SCALAR_DTYPES'
]

# NDArray value dtype id <-> name (encodings.py:131-143) and shape dtype ids (:114-119).
VALUE_DTYPES = {
    8: 'uint8',
    9: 'int8',
    16: 'uint16',
    17: 'int16',
    18: 'float16',
    32: 'uint32',
    33: 'int32',
    34: 'float32',
    64: 'uint64',
    65: 'int64',
    66: 'float64',
}
_VALUE_DTYPE_IDS = {v: k for k, v in VALUE_DTYPES.items()}
_SHAPE_DTYPES = {0: 'uint8', 1: 'uint16', 2: 'uint32', 3: 'uint64'}

SCALAR_DTYPES = ('uint8', 'uint16', 'uint32', 'uint64', 'int8', 'int16', 'int32', 'int64',
                 'float16', 'float32', 'float64')

_HOST_OBJECT = ('str_int', 'str_float', 'str_decimal', 'pil', 'jpeg', 'jpeg_array', 'jpegarray',
                'png', 'list[pil]', 'list[jpeg]', 'list[png]', 'pkl', 'json')

_NAMES = frozenset(('bytes', 'str', 'int', 'ndarray') + SCALAR_DTYPES + _HOST_OBJECT)
_UNSAFE = frozenset(('pkl',))


@dataclass(frozen=True)
class EncodingInfo:
    """What an encoding string means.

    Attributes:
        name: registry name (``bytes``, ``str``, ``int``, ``ndarray``, ``float32``, ``pil`` ...).
        dtype: numpy dtype name for scalars and ndarrays with a static dtype, else None.
        shape: static ndarray shape, or ``()`` for scalars / ``int``, else None.
        size: fixed encoded size in bytes, or None if variable (``get_mds_encoded_size``).
    """
    name: str
    dtype: Optional[str]
    shape: Optional[tuple[int, ...]]
    size: Optional[int]

    @property
    def is_host_object(self) -> bool:
        return self.name in _HOST_OBJECT


def _py_int(text: str) -> int:
    return int(text)  # Python's own int() grammar, as NDArray.from_str uses (encodings.py:191)


def parse_encoding(encoding: str) -> Optional[EncodingInfo]:
    """Parse an encoding string like ``_get_coder`` (encodings.py:697-714); None if unknown.

    Raises the reference's exception types for malformed ``ndarray:`` configs.
    """
    index = encoding.find(':')
    if index == -1:
        if encoding not in _NAMES:
            return None
        if encoding == 'int':
            return EncodingInfo('int', 'int64', (), 8)
        if encoding in SCALAR_DTYPES:
            return EncodingInfo(encoding, encoding, (), np.dtype(encoding).itemsize)
        return EncodingInfo(encoding, None, None, None)
    name, config = encoding[:index], encoding[index + 1:]
    if name not in _NAMES:
        raise KeyError(name)
    if name != 'ndarray':
        raise AttributeError(f'{name} has no from_str')
    args = config.split(':') if config else []
    if len(args) not in (0, 1, 2):
        raise AssertionError(f'bad ndarray encoding {encoding!r}')
    dtype = args[0] if len(args) >= 1 else None
    shape = tuple(map(_py_int, args[1].split(','))) if len(args) >= 2 else None
    if dtype is not None and dtype not in _VALUE_DTYPE_IDS:
        raise AssertionError(f'bad ndarray dtype {dtype!r}')
    if shape is not None and any(d < 1 for d in shape):
        raise AssertionError(f'bad ndarray shape {shape!r}')
    size = None
    if dtype is not None and shape is not None:
        size = int(np.prod(shape)) * np.dtype(dtype).itemsize
    return EncodingInfo('ndarray', dtype, shape, size)


def get_mds_encodings() -> set[str]:
    """Supported encoding names (encodings.py:717-723)."""
    return set(_NAMES)


def is_mds_encoding(encoding: str) -> bool:
    """Whether the encoding is supported (encodings.py:726-735)."""
    try:
        return parse_encoding(encoding) is not None
    except (KeyError, AttributeError, AssertionError, ValueError):
        return False


def is_mds_encoding_safe(encoding: str) -> bool:
    """Whether the encoding cannot run code when decoded (encodings.py:730-739)."""
    return encoding not in _UNSAFE


def get_mds_encoded_size(encoding: str) -> Optional[int]:
    """Fixed encoded size, or None (encodings.py:776-788)."""
    info = parse_encoding(encoding)
    if info is None:
        raise ValueError(f'Unsupported encoding: {encoding}.')
    return info.size


# ---------------------------------------------------------------------------------------------
# Encode (writer side).


def _require(obj: Any, expected: Any) -> None:
    if not isinstance(obj, expected):
        raise AttributeError(f'data should be of type {expected}, but instead, found as {type(obj)}')


def _encode_ndarray(info: EncodingInfo, obj: np.ndarray) -> bytes:
    # Layout of NDArray.encode (encodings.py:215-268):
    # [dtype id: u8 if dynamic dtype][ndim<<2 | shape dtype: u8, shape if dynamic shape][values]
    parts = []
    dtype_id = _VALUE_DTYPE_IDS.get(obj.dtype.name)
    if dtype_id is None:
        raise ValueError(f'Unsupported dtype: {obj.dtype.name}.')
    if info.dtype is None:
        parts.append(bytes([dtype_id]))
    elif obj.dtype != info.dtype:
        raise ValueError(f'Wrong dtype: expected {info.dtype}, got {obj.dtype.name}.')
    if obj.size == 0:
        raise ValueError('Attempting to encode a numpy array with 0 elements.')
    if info.shape is None:
        ndim = obj.ndim
        if ndim >= 64:
            raise ValueError('Array has too many axes: maximum 63, got {ndim}.')
        if ndim == 0:
            raise ValueError('Attempting to encode a scalar with NDArray encoding. Please use a '
                             'scalar encoding.')
        shape = np.array(obj.shape, np.int64)
        if shape.min() <= 0:
            raise ValueError('All dimensions must be greater than zero.')
        top = int(shape.max())
        code = 0 if top < (1 << 8) else 1 if top < (1 << 16) else 2 if top < (1 << 32) else 3
        parts.append(bytes([(ndim << 2) | code]))
        parts.append(shape.astype(_SHAPE_DTYPES[code]).tobytes())
    elif obj.shape != info.shape:
        raise ValueError(f'Wrong shape: expected {info.shape}, got {obj.shape}.')
    parts.append(obj.tobytes())
    return b''.join(parts)


def _encode_list(element_encode, obj: list) -> bytes:
    # List layout (encodings.py:556-575): [u32 0][u32 n][n x u32 sizes][elements]
    _require(obj, list)
    elems = [element_encode(x) for x in obj]
    head = np.array([0, len(elems)] + [len(x) for x in elems], np.uint32).tobytes()
    return head + b''.join(elems)


def _encode_pil(obj: Any) -> bytes:
    from PIL import Image
    _require(obj, Image.Image)
    mode = obj.mode.encode('utf-8')
    width, height = obj.size
    return np.array([width, height, len(mode)], np.uint32).tobytes() + mode + obj.tobytes()


def _encode_image(obj: Any, fmt: str) -> bytes:
    from PIL import Image
    _require(obj, Image.Image)
    if fmt == 'JPEG':
        from PIL.JpegImagePlugin import JpegImageFile
        filename = getattr(obj, 'filename', None)
        if isinstance(obj, JpegImageFile) and filename:
            try:
                with open(filename, 'rb') as f:
                    return f.read()
            except FileNotFoundError:
                pass
    out = BytesIO()
    obj.save(out, format=fmt)
    return out.getvalue()


def mds_encode(encoding: str, obj: Any) -> bytes:
    """Encode one value (encodings.py:742-757): ``bytes`` pass through for every encoding."""
    if isinstance(obj, bytes):
        return obj
    info = parse_encoding(encoding)
    if info is None:
        raise ValueError(f'Unsupported encoding: {encoding}.')
    name = info.name
    if name == 'bytes':
        _require(obj, bytes)
    if name == 'str':
        _require(obj, str)
        return obj.encode('utf-8')
    if name == 'int':
        _require(obj, int)
        return np.int64(obj).tobytes()
    if name in SCALAR_DTYPES:
        return np.dtype(name).type(obj).tobytes()
    if name == 'ndarray':
        return _encode_ndarray(info, obj)
    if name == 'str_int':
        _require(obj, int)
        return str(obj).encode('utf-8')
    if name == 'str_float':
        _require(obj, float)
        return str(obj).encode('utf-8')
    if name == 'str_decimal':
        _require(obj, Decimal)
        return str(obj).encode('utf-8')
    if name == 'pil':
        return _encode_pil(obj)
    if name == 'jpeg':
        return _encode_image(obj, 'JPEG')
    if name == 'png':
        return _encode_image(obj, 'PNG')
    if name == 'list[pil]':
        return _encode_list(_encode_pil, obj)
    if name == 'list[jpeg]':
        return _encode_list(lambda x: _encode_image(x, 'JPEG'), obj)
    if name == 'list[png]':
        return _encode_list(lambda x: _encode_image(x, 'PNG'), obj)
    if name in ('jpeg_array', 'jpegarray'):
        # [u32 n][n x u32 sizes][images] (encodings.py:612-620)
        sizes = [len(x) for x in obj]
        return np.uint32(len(obj)).tobytes() + np.array(sizes, np.uint32).tobytes() + b''.join(
            bytes(x) for x in obj)
    if name == 'pkl':
        return pickle.dumps(obj)
    if name == 'json':
        if isinstance(obj, np.ndarray):
            obj = obj.tolist()
        text = json.dumps(obj)
        json.loads(text)
        return text.encode('utf-8')
    raise ValueError(f'Unsupported encoding: {encoding}.')  # pragma: no cover


# ---------------------------------------------------------------------------------------------
# Host-side object construction over device-gathered bytes.


def ndarray_dyn_decode(info: EncodingInfo, data: bytes) -> np.ndarray:
    """Split a dynamic ndarray's header and view its values (encodings.py:270-305)."""
    index = 0
    if info.dtype:
        dtype = info.dtype
    else:
        dtype = VALUE_DTYPES[data[index]]
        index += 1
    if info.shape:
        shape = info.shape
    else:
        byte = data[index]
        index += 1
        ndim, code = byte >> 2, byte % 4
        nbytes = ndim * (1 << code)
        shape = np.frombuffer(data[index:index + nbytes], _SHAPE_DTYPES[code])
        index += nbytes
    return np.frombuffer(data[index:], dtype).reshape(shape)


def _decode_pil(data: bytes) -> Any:
    from PIL import Image
    width, height, mode_size = np.frombuffer(data[:12], np.uint32)
    mode = data[12:12 + mode_size].decode('utf-8')
    return Image.frombytes(mode, (width, height), data[12 + mode_size:])


def _decode_image(data: bytes) -> Any:
    from PIL import Image
    return Image.open(BytesIO(data))


def _decode_list(element_decode, data: bytes) -> list:
    num = int(np.frombuffer(data[4:8], np.uint32)[0])
    sizes = np.frombuffer(data[8:8 + 4 * num], np.uint32)
    index = 8 + 4 * num
    out = []
    for size in sizes:
        out.append(element_decode(data[index:index + size]))
        index += int(size)
    return out


def _decode_jpeg_array(data: bytes) -> list:
    if len(data) < 4:
        raise ValueError('Input data is too short to contain valid jpeg arrays')
    n = int(np.frombuffer(data[:4], np.uint32)[0])
    if n <= 0:
        raise ValueError('Negative number of images decoded')
    start = 4 + 4 * n
    if len(data) < start:
        raise ValueError('Data is too short w.r.t the number of images decoded')
    sizes = np.frombuffer(data[4:start], np.uint32).tolist()
    out, lo = [], start
    for size in sizes:
        out.append(_decode_image(data[lo:lo + size]))
        lo += size
    return out


def host_object_decode(encoding: str, data: bytes) -> Any:
    """Python object of a host-object encoding from its (device-gathered) bytes."""
    info = parse_encoding(encoding)
    if info is None:
        raise ValueError(f'Unsupported encoding: {encoding}.')
    name = info.name
    if name == 'str_int':
        return int(data.decode('utf-8'))
    if name == 'str_float':
        return float(data.decode('utf-8'))
    if name == 'str_decimal':
        return Decimal(data.decode('utf-8'))
    if name == 'pil':
        return _decode_pil(data)
    if name in ('jpeg', 'png'):
        return _decode_image(data)
    if name == 'list[pil]':
        return _decode_list(_decode_pil, data)
    if name in ('list[jpeg]', 'list[png]'):
        return _decode_list(_decode_image, data)
    if name in ('jpeg_array', 'jpegarray'):
        return _decode_jpeg_array(data)
    if name == 'pkl':
        return pickle.loads(data)
    if name == 'json':
        return json.loads(data.decode('utf-8'))
    raise ValueError(f'{encoding} is decoded on the device, not by host_object_decode')
