"""Drop-in plugin for mosaicml/streaming's ``StreamingDataset``.

``StreamingDataset(stream_name=..., stream_config=...)`` builds its streams through the public
``streams_registry`` (``streaming/base/stream.py:515-522``, used at
``streaming/base/dataset.py:447-468``). :func:`make_device_stream` derives a ``Stream`` class whose
``get_shards`` (``stream.py:428-484``: index download/parse, ``reader_from_json``, ``validate``) is
the reference's own, with each MDS reader swapped for :class:`streaming_amd.reader.MDSReader`
(same ``Reader`` interface; samples decoded on the GPU a whole shard at a time). Readers of other
formats (JSONL, CSV) are returned unchanged.
"""

from __future__ import annotations

from typing import Any, Optional, Union

import torch

from streaming_amd.reader import FileInfo, MDSReader

__all__ = ['to_device_reader', 'make_device_stream', 'register_device_stream']


def _file_info(f: Any) -> Optional[FileInfo]:
    if f is None:
        return None
    return FileInfo(f.basename, f.bytes, dict(f.hashes))


def to_device_reader(reader: Any, device: Union[str, torch.device, None] = None) -> Any:
    """The device-backed equivalent of a reference ``MDSReader`` (other readers unchanged)."""
    if isinstance(reader, MDSReader) or getattr(reader, 'column_encodings', None) is None:
        return reader
    return MDSReader(dirname=reader.dirname,
                     split=reader.split or None,
                     column_encodings=list(reader.column_encodings),
                     column_names=list(reader.column_names),
                     column_sizes=list(reader.column_sizes),
                     compression=reader.compression,
                     hashes=list(reader.hashes),
                     raw_data=_file_info(reader.raw_data),
                     samples=reader.samples,
                     size_limit=reader.size_limit,
                     zip_data=_file_info(reader.zip_data),
                     device=device)


def make_device_stream(stream_base: type, device: Union[str, torch.device, None] = None) -> type:
    """A subclass of the reference ``Stream`` whose shards decode on the GPU."""

    class DeviceStream(stream_base):  # type: ignore[misc, valid-type]
        """``Stream`` with MI355X-decoded MDS shards (``streaming_amd``)."""

        def get_shards(self, world: Any, allow_unsafe_types: bool) -> list:
            shards = super().get_shards(world, allow_unsafe_types)
            return [to_device_reader(s, device) for s in shards]

    DeviceStream.__name__ = 'DeviceStream'
    DeviceStream.__qualname__ = 'DeviceStream'
    return DeviceStream


def register_device_stream(name: str = 'mdsx',
                           device: Union[str, torch.device, None] = None) -> type:
    """Register the device stream in the reference's ``streams_registry`` under ``name``."""
    from streaming.base.stream import Stream, streams_registry  # the reference package
    cls = make_device_stream(Stream, device)
    streams_registry.register(name, func=cls)
    return cls
