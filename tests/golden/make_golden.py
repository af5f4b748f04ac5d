"""Generate the golden MDS fixtures under tests/golden/ with the REAL reference.

Run in the build container only (the reference is at /root/reference there and nowhere else):

    python tests/golden/make_golden.py [--reference /root/reference]

It imports mosaicml/streaming offline -- optional codec/registry packages that are not installed
(brotli, snappy, zstd, catalogue) are replaced by small stubs written to a temporary directory
(zstd binds the system libzstd through ctypes), the model-zoo subpackages are preset to empty
modules, and bytecode writing is disabled so nothing is written into the reference tree. Then
for every dataset below it:

1. writes the shards with the reference ``MDSWriter`` into ``tests/golden/<name>/``;
2. reads every sample back with the reference ``reader_from_json(...)[i]``;
3. records the reference's decoded values (``items.json``, small sets) and, in the device
   decoder's output format, the expected columns (``expected.npz``, small sets) and their sha256
   digests (``manifest.json``, every set).

For ``str`` rows the reference cannot decode (invalid UTF-8 raises ``UnicodeDecodeError``) the
expected bytes come from the same reference reader with that column's encoding read as
``bytes``, and the expected flag is 1.
"""

from __future__ import annotations

import argparse
import hashlib
import importlib
import json
import os
import shutil
import sys
import tempfile
import types
from decimal import Decimal

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

_STUB_ZSTD = r'''
import ctypes, ctypes.util
_z = ctypes.CDLL(ctypes.util.find_library('zstd') or 'libzstd.so.1')
_z.ZSTD_compressBound.restype = ctypes.c_size_t
_z.ZSTD_compressBound.argtypes = [ctypes.c_size_t]
_z.ZSTD_compress.restype = ctypes.c_size_t
_z.ZSTD_compress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
_z.ZSTD_decompress.restype = ctypes.c_size_t
_z.ZSTD_decompress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
_z.ZSTD_getFrameContentSize.restype = ctypes.c_ulonglong
_z.ZSTD_getFrameContentSize.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
_z.ZSTD_isError.restype = ctypes.c_uint
_z.ZSTD_isError.argtypes = [ctypes.c_size_t]
def compress(data, level=3):
    bound = _z.ZSTD_compressBound(len(data))
    out = ctypes.create_string_buffer(bound)
    n = _z.ZSTD_compress(out, bound, data, len(data), level)
    assert not _z.ZSTD_isError(n)
    return out.raw[:n]
def decompress(data):
    size = _z.ZSTD_getFrameContentSize(data, len(data))
    out = ctypes.create_string_buffer(max(size, 1))
    n = _z.ZSTD_decompress(out, size, data, len(data))
    assert not _z.ZSTD_isError(n)
    return out.raw[:n]
'''

_STUB_UNAVAILABLE = '''
def compress(*args, **kwargs):
    raise NotImplementedError('not installed in this image')
def decompress(*args, **kwargs):
    raise NotImplementedError('not installed in this image')
'''

_STUB_CATALOGUE = '''
REGISTRY = {}
class RegistryError(Exception):
    pass
class Registry:
    def __init__(self, *namespace, entry_points=False):
        self.namespace = namespace
        self._d = {}
    def register(self, name, func=None):
        if func is None:
            def deco(f):
                self._d[name] = f
                return f
            return deco
        self._d[name] = func
        return func
    def get(self, name):
        if name not in self._d:
            raise RegistryError(name)
        return self._d[name]
    def get_all(self):
        return dict(self._d)
    def get_entry_points(self):
        return {}
    def get_entry_point(self, name, default=None):
        return default
    def find(self, name):
        return {}
def create(*namespace, entry_points=False):
    return Registry(*namespace, entry_points=entry_points)
def check_exists(*namespace):
    return False
'''


def boot_reference(ref: str):
    sys.dont_write_bytecode = True
    stub = tempfile.mkdtemp(prefix='refstubs_')
    for name, text in (('zstd', _STUB_ZSTD), ('brotli', _STUB_UNAVAILABLE),
                       ('snappy', _STUB_UNAVAILABLE), ('catalogue', _STUB_CATALOGUE)):
        with open(os.path.join(stub, f'{name}.py'), 'w') as f:
            f.write(text)
    sys.path.insert(0, stub)
    for m in ('streaming.vision', 'streaming.text', 'streaming.multimodal'):
        sys.modules[m] = types.ModuleType(m)
    sys.path.insert(0, ref)
    import streaming  # noqa: F401
    from streaming.base.format import reader_from_json
    from streaming.base.format.mds import MDSWriter
    from streaming.base.format.mds.encodings import mds_decode
    return MDSWriter, reader_from_json, mds_decode


# ---------------------------------------------------------------------------------------------
# Dataset generators (deterministic).


def random_text(rng: np.random.Generator, lo: int, hi: int) -> str:
    """Code points mixing 1/2/3/4-byte UTF-8 (no surrogates)."""
    n = int(rng.integers(lo, hi + 1))
    width = rng.integers(0, 4, n)
    cps = []
    for w in width:
        if w == 0:
            cps.append(int(rng.integers(0x20, 0x7F)))
        elif w == 1:
            cps.append(int(rng.integers(0x80, 0x800)))
        elif w == 2:
            cp = int(rng.integers(0x800, 0x10000 - 0x800))
            cps.append(cp + 0x800 if cp >= 0xD800 else cp)
        else:
            cps.append(int(rng.integers(0x10000, 0x110000)))
    return ''.join(map(chr, cps))


def gen_kat():
    cols = {'s': 'str', 'a': 'int', 'b': 'bytes'}
    samples = [{'s': 'hé', 'a': -2, 'b': b'\x00\x01\x02'}, {'s': '', 'a': 7, 'b': b''}]
    return cols, samples, {}


def gen_config_a(ref: str):
    sys.path.insert(0, os.path.join(ref, 'regression'))
    mod = importlib.import_module('synthetic_dataset')
    ds = mod.NumberAndSayDataset(num_samples=10_000, seed=987)
    samples = list(ds)
    return {'number': 'int', 'words': 'str'}, samples, {'size_limit': 10240}


def gen_config_a2(ref: str):
    """A second stream of config A's schema (multi-stream loader order, make_loader_fixtures)."""
    sys.path.insert(0, os.path.join(ref, 'regression'))
    mod = importlib.import_module('synthetic_dataset')
    ds = mod.NumberAndSayDataset(num_samples=3_000, seed=4242)
    samples = list(ds)
    return {'number': 'int', 'words': 'str'}, samples, {'size_limit': 10240}


def gen_sequence():
    samples = [{'id': f'{i:06}', 'sample': 3 * i} for i in range(117)]
    return {'id': 'str', 'sample': 'int'}, samples, {'size_limit': 1 << 8}


def gen_config_b_small():
    rng = np.random.default_rng(0)
    n = 250
    x = rng.integers(0, 2**32, (n, 1024), dtype=np.uint32)
    x[0, :4] = [0x7fc00001, 0xffc00000, 0x7f800000, 0x00000001]  # NaN payloads, inf, denormal
    xf = x.view(np.float32)
    samples = [{'id': np.int32(i - 7), 'x': xf[i]} for i in range(n)]
    return {'id': 'int32', 'x': 'ndarray:float32:1024'}, samples, {'size_limit': 1 << 19}


def gen_config_c_small():
    rng = np.random.default_rng(1)
    samples = []
    for _ in range(200):
        samples.append({
            'n': int(rng.integers(-2**62, 2**62)),
            'b': rng.bytes(int(rng.integers(3072, 5121))),
            's': random_text(rng, 16, 256),
        })
    return {'n': 'int', 'b': 'bytes', 's': 'str'}, samples, {'size_limit': 1 << 19}


_SCALAR_COLS = {
    'u8': 'uint8',
    'u16': 'uint16',
    'u32': 'uint32',
    'u64': 'uint64',
    'i8': 'int8',
    'i16': 'int16',
    'i32': 'int32',
    'i64': 'int64',
    'f16': 'float16',
    'f32': 'float32',
    'f64': 'float64',
    'n': 'int',
    'a3': 'ndarray:uint8:3',
    'a7': 'ndarray:float16:7',
    'a23': 'ndarray:int16:2,3',
    'a5': 'ndarray:float64:5',
    'a4': 'ndarray:uint32:4',
    'a17': 'ndarray:int8:17',
    'a11': 'ndarray:uint16:1,1',
    'a300': 'ndarray:int32:300',
    'a6x7': 'ndarray:uint8:6,7',
}


def gen_scalars():
    rng = np.random.default_rng(2)
    samples = []
    for i in range(120):
        s = {}
        for name, enc in _SCALAR_COLS.items():
            if enc == 'int':
                s[name] = int(rng.integers(-2**63, 2**63 - 1))
            elif enc.startswith('ndarray'):
                _, dtype, shape = enc.split(':')
                shape = tuple(int(d) for d in shape.split(','))
                nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
                s[name] = np.frombuffer(rng.bytes(nbytes), dtype).reshape(shape)
            else:
                s[name] = np.frombuffer(rng.bytes(np.dtype(enc).itemsize), enc)[0]
        samples.append(s)
    return _SCALAR_COLS, samples, {'size_limit': 1 << 13}


def gen_dynamic():
    rng = np.random.default_rng(3)
    dtypes = ['uint8', 'int8', 'uint16', 'int16', 'float16', 'uint32', 'int32', 'float32',
              'uint64', 'int64', 'float64']
    samples = []
    for i in range(200):
        ndim = int(rng.integers(1, 4))
        shape = tuple(int(rng.integers(1, 6)) for _ in range(ndim))
        if i % 17 == 0:
            shape = (300, 1)  # uint16 shape dtype
        dt = dtypes[i % len(dtypes)]
        count = int(np.prod(shape))
        a0 = np.frombuffer(rng.bytes(count * np.dtype(dt).itemsize), dt).reshape(shape)
        a1 = rng.integers(-1000, 1000, shape).astype(np.int16)
        a2 = rng.standard_normal(shape).astype(np.float32)
        samples.append({
            'd0': a0,
            'd1': a1,
            'd2': a2,
            'j': {'i': i, 'v': [float(rng.standard_normal()), None, 'x' * (i % 5)]},
            'si': int(rng.integers(-10**15, 10**15)) * 10**15 + int(rng.integers(0, 10**15)),
            'sf': float(rng.standard_normal()),
            'sd': Decimal(int(rng.integers(-10**9, 10**9))) / Decimal(1000),
            'e': rng.bytes(int(rng.integers(0, 40))) if i % 3 else b'',
        })
    cols = {
        'd0': 'ndarray',
        'd1': 'ndarray:int16',
        'd2': 'ndarray:float32',
        'j': 'json',
        'si': 'str_int',
        'sf': 'str_float',
        'sd': 'str_decimal',
        'e': 'bytes'
    }
    return cols, samples, {'size_limit': 1 << 14}


def gen_images():
    from PIL import Image
    rng = np.random.default_rng(4)
    samples = []
    for i in range(10):
        w, h = int(rng.integers(2, 9)), int(rng.integers(2, 9))
        arr = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        img = Image.fromarray(arr, 'RGB')
        gray = Image.fromarray(arr[:, :, 0], 'L')
        from io import BytesIO
        buf = BytesIO()
        img.save(buf, format='JPEG')
        samples.append({
            'p': img,
            'g': gray,
            'lp': [gray, gray],
            'ja': [buf.getvalue(), buf.getvalue()],
        })
    return {'p': 'pil', 'g': 'png', 'lp': 'list[png]', 'ja': 'jpeg_array'}, samples, {}


BAD_UTF8 = [
    b'plain ascii',
    b'',
    'héllo € \U0001F600'.encode(),
    b'\x80',  # lone continuation
    b'abc\xbf',  # trailing lone continuation
    b'\xc0\xaf',  # overlong 2-byte
    b'\xc1\xbf',  # overlong 2-byte
    b'\xe0\x80\xaf',  # overlong 3-byte
    b'\xe0\xa0\x80',  # smallest valid 3-byte (U+0800)
    b'\xed\xa0\x80',  # surrogate U+D800
    b'\xed\x9f\xbf',  # U+D7FF valid
    b'\xee\x80\x80',  # U+E000 valid
    b'\xf0\x80\x80\x80',  # overlong 4-byte
    b'\xf0\x90\x80\x80',  # U+10000 valid
    b'\xf4\x8f\xbf\xbf',  # U+10FFFF valid
    b'\xf4\x90\x80\x80',  # > U+10FFFF
    b'\xf5\x80\x80\x80',  # invalid lead
    b'\xff',  # invalid byte
    b'ok\xc3',  # truncated 2-byte at end
    b'ok\xe2\x82',  # truncated 3-byte at end
    b'ok\xf0\x9f\x98',  # truncated 4-byte at end
    b'\xc3\x28',  # bad continuation
    b'\xe2\x28\xa1',  # bad continuation
    b'x' * 15 + b'\xc3\xa9' + b'y' * 40,  # 2-byte across a 16-byte chunk boundary
    b'x' * 14 + b'\xe2\x82\xac' + b'y' * 40,  # 3-byte across a chunk boundary
    b'x' * 13 + b'\xf0\x9f\x98\x80' + b'y' * 40,  # 4-byte across a chunk boundary
    b'x' * 15 + b'\xc3' + b'y' * 40,  # truncated at a chunk boundary
    b'x' * 16 + b'\x80' + b'y' * 40,  # lone continuation at a chunk start
    'é'.encode() * 600,  # long valid 2-byte text
    'é'.encode() * 600 + b'\x80',  # long text, bad at the end
    b'\xe0' + 'é'.encode() * 300,  # bad at the start of a long row
    '\U0001F600'.encode() * 100 + b'\xed\xbf\xbf' + b'z' * 1000,  # surrogate in the middle
]


def gen_bad_utf8():
    samples = [{'s': data, 'k': i} for i, data in enumerate(BAD_UTF8)]
    return {'s': 'str', 'k': 'int'}, samples, {}


def gen_zstd():
    rng = np.random.default_rng(5)
    n = 100
    x = rng.integers(0, 256, (n, 1024)).astype(np.float32)
    samples = [{'id': np.int32(i), 'x': x[i]} for i in range(n)]
    return {'id': 'int32', 'x': 'ndarray:float32:1024'}, samples, {
        'size_limit': 1 << 18,
        'compression': 'zstd',
        'hashes': ['sha1', 'xxh64']
    }


def gen_zstd_xxh3():
    # ragged columns, zstd, and the xxh3 digests the pipeline validates on the device
    rng = np.random.default_rng(6)
    samples = []
    for _ in range(120):
        blob = rng.integers(0, 8, int(rng.integers(500, 3000))).astype(np.uint8).tobytes()
        samples.append({'n': int(rng.integers(-2**62, 2**62)), 'b': blob,
                        's': random_text(rng, 5, 40)})
    return {'n': 'int', 'b': 'bytes', 's': 'str'}, samples, {
        'size_limit': 1 << 17,
        'compression': 'zstd',
        'hashes': ['xxh128', 'xxh3_64']
    }


def gen_wide():
    rng = np.random.default_rng(6)
    cols = {}
    for k in range(20):
        cols[f'v{k:02}'] = 'bytes' if k % 2 else 'str'
        cols[f'f{k:02}'] = ['int', 'float32', 'ndarray:uint8:5', 'ndarray:int16:40'][k % 4]
    samples = []
    for i in range(300):
        s = {}
        for name, enc in cols.items():
            if enc == 'bytes':
                s[name] = rng.bytes(int(rng.integers(0, 60)))
            elif enc == 'str':
                s[name] = random_text(rng, 0, 20)
            elif enc == 'int':
                s[name] = int(rng.integers(-2**40, 2**40))
            elif enc == 'float32':
                s[name] = np.float32(rng.standard_normal())
            elif enc == 'ndarray:uint8:5':
                s[name] = rng.integers(0, 256, 5, dtype=np.uint8)
            else:
                s[name] = rng.integers(-999, 999, 40).astype(np.int16)
        samples.append(s)
    return cols, samples, {'size_limit': 1 << 15}


# ---------------------------------------------------------------------------------------------


def value_record(v) -> dict:
    """JSON record of a reference-decoded value (type + exact content)."""
    from PIL import Image
    if isinstance(v, bool):
        raise TypeError('unexpected bool')
    if isinstance(v, int):
        return {'t': 'int', 'v': str(v)}
    if isinstance(v, float):
        return {'t': 'float', 'v': v.hex()}
    if isinstance(v, Decimal):
        return {'t': 'Decimal', 'v': str(v)}
    if isinstance(v, bytes):
        return {'t': 'bytes', 'hex': v.hex()}
    if isinstance(v, str):
        return {'t': 'str', 'v': v}
    if isinstance(v, np.ndarray):
        return {
            't': 'ndarray',
            'dtype': v.dtype.name,
            'shape': list(v.shape),
            'hex': v.tobytes().hex(),
            'writeable': bool(v.flags.writeable)
        }
    if isinstance(v, np.generic):
        return {'t': 'np', 'dtype': v.dtype.name, 'hex': v.tobytes().hex()}
    if isinstance(v, Image.Image):
        return {'t': 'PIL', 'mode': v.mode, 'size': list(v.size), 'hex': v.tobytes().hex()}
    if isinstance(v, list):
        return {'t': 'list', 'items': [value_record(x) for x in v]}
    if isinstance(v, dict):
        return {'t': 'json', 'v': v}
    raise TypeError(f'unexpected value type {type(v)}')


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument('--reference', default='/root/reference')
    ap.add_argument('--only', default='')
    args = ap.parse_args()
    MDSWriter, reader_from_json, ref_decode = boot_reference(args.reference)

    specs = {
        'kat': (gen_kat, True),
        'config_a': (lambda: gen_config_a(args.reference), False),
        'config_a2': (lambda: gen_config_a2(args.reference), False),
        'sequence': (gen_sequence, True),
        'config_b_small': (gen_config_b_small, False),
        'config_c_small': (gen_config_c_small, False),
        'scalars': (gen_scalars, True),
        'dynamic': (gen_dynamic, True),
        'images': (gen_images, True),
        'bad_utf8': (gen_bad_utf8, True),
        'zstd': (gen_zstd, False),
        'zstd_xxh3': (gen_zstd_xxh3, False),
        'wide': (gen_wide, False),
    }
    manifest_path = os.path.join(HERE, 'manifest.json')
    manifest = {}
    if os.path.exists(manifest_path):
        with open(manifest_path) as f:
            manifest = json.load(f)
    only = set(filter(None, args.only.split(',')))
    for name, (gen, keep_items) in specs.items():
        if only and name not in only:
            continue
        cols, samples, kwargs = gen()
        out = os.path.join(HERE, name)
        shutil.rmtree(out, ignore_errors=True)
        with MDSWriter(columns=cols, out=out, **kwargs) as w:
            for s in samples:
                w.write(s)
        with open(os.path.join(out, 'index.json')) as f:
            index = json.load(f)
        if kwargs.get('compression'):  # the reference reads raw files: decompress them here
            from streaming.base.compression import decompress
            for info in index['shards']:
                with open(os.path.join(out, info['zip_data']['basename']), 'rb') as f:
                    raw = decompress(info['compression'], f.read())
                with open(os.path.join(out, info['raw_data']['basename']), 'wb') as f:
                    f.write(raw)
        entry = {'shards': [], 'columns': {}}
        items = []
        npz = {}
        per_col = {c: [] for c in index['shards'][0]['column_names']}
        for si, info in enumerate(index['shards']):
            reader = reader_from_json(out, None, info)
            as_bytes = dict(info)  # the same reference reader, every column read as raw bytes
            as_bytes['column_encodings'] = ['bytes'] * len(info['column_encodings'])
            raw_reader = reader_from_json(out, None, as_bytes)
            with open(os.path.join(out, info['raw_data']['basename']), 'rb') as f:
                shard_bytes = f.read()
            entry['shards'].append({
                'basename': info['raw_data']['basename'],
                'samples': info['samples'],
                'sha256': hashlib.sha256(shard_bytes).hexdigest()
            })
            for i in range(info['samples']):
                raw = raw_reader[i]
                try:
                    full = reader[i]
                except UnicodeDecodeError:
                    full = None
                rec = {}
                for c, enc, size in zip(info['column_names'], info['column_encodings'],
                                        info['column_sizes']):
                    bad = False
                    try:
                        value = ref_decode(enc, raw[c])
                    except UnicodeDecodeError:
                        bad, value = True, None
                    if full is not None and keep_items:
                        assert value_record(full[c]) == value_record(value), (name, i, c)
                    if keep_items:
                        rec[c] = {'t': 'error', 'exc': 'UnicodeDecodeError'} if bad else \
                            value_record(value)
                    if size:
                        if isinstance(value, (np.ndarray, np.generic)):
                            assert value.tobytes() == raw[c], (name, i, c)
                        elif enc == 'int':
                            assert np.int64(value).tobytes() == raw[c], (name, i, c)
                        assert len(raw[c]) == size, (name, c, len(raw[c]), size)
                        per_col[c].append(('fixed', raw[c], None))
                    else:
                        if enc == 'bytes':
                            assert value == raw[c]
                        per_col[c].append(('ragged', raw[c], bad if enc == 'str' else None))
                if keep_items:
                    items.append(rec)
            # release file handles promptly
            del reader, raw_reader
        for c, vals in per_col.items():
            if vals[0][0] == 'fixed':
                arr = np.frombuffer(b''.join(v[1] for v in vals), np.uint8).reshape(len(vals), -1)
                npz[f'{c}.rows'] = arr
                entry['columns'][c] = {'rows': hashlib.sha256(arr.tobytes()).hexdigest()}
            else:
                lens = np.array([len(v[1]) for v in vals], np.int64)
                offsets = np.concatenate([np.zeros(1, np.int64), np.cumsum(lens)])
                values = np.frombuffer(b''.join(v[1] for v in vals), np.uint8)
                npz[f'{c}.values'] = values
                npz[f'{c}.offsets'] = offsets
                d = {
                    'values': hashlib.sha256(values.tobytes()).hexdigest(),
                    'offsets': hashlib.sha256(offsets.tobytes()).hexdigest()
                }
                if vals[0][2] is not None:
                    flags = np.array([1 if v[2] else 0 for v in vals], np.uint8)
                    npz[f'{c}.flags'] = flags
                    d['flags'] = hashlib.sha256(flags.tobytes()).hexdigest()
                entry['columns'][c] = d
        if keep_items:
            np.savez_compressed(os.path.join(out, 'expected.npz'), **npz)
            with open(os.path.join(out, 'items.json'), 'w') as f:
                json.dump(items, f)
        if kwargs.get('compression'):  # keep only the compressed files, as the writer left them
            for info in index['shards']:
                os.remove(os.path.join(out, info['raw_data']['basename']))
        entry['rows'] = sum(s['samples'] for s in entry['shards'])
        manifest[name] = entry
        print(f'{name}: {len(index["shards"])} shards, {entry["rows"]} samples', flush=True)

    if not only or 'config_a' in only:
        # Ordered content digest of config A: (int64 number, utf8 words).
        h = hashlib.sha256()
        idx = json.load(open(os.path.join(HERE, 'config_a', 'index.json')))
        for info in idx['shards']:
            r = reader_from_json(os.path.join(HERE, 'config_a'), None, info)
            for i in range(info['samples']):
                s = r[i]
                h.update(np.int64(s['number']).tobytes())
                h.update(s['words'].encode('utf-8'))
        manifest['config_a']['content_sha256'] = h.hexdigest()
    with open(manifest_path, 'w') as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == '__main__':
    main()
