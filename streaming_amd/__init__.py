"""streaming_amd: MI355X-native MDS shard decoder for mosaicml/streaming's MDS format.

The hot path -- offsets-table scan, per-sample byte-range gather and per-column decode over
whole shards -- runs as hand-written gfx950 HIP kernels in ``libmdsx.so`` (C ABI:
``include/mdsx.h``). The Python layer mirrors the reference's ``Reader`` / ``MDSReader`` /
``LocalDataset`` / ``MDSWriter`` interfaces.
"""

from streaming_amd.array import Array
from streaming_amd.decoder import (BatchDecoder, DecodedBatch, DeviceBatch, Plan, RaggedColumn,
                                   decode_batch, stage_shards)
from streaming_amd.local import LocalDataset, shard_assignment
from streaming_amd.reader import FileInfo, JointReader, MDSReader, Reader, reader_from_json
from streaming_amd.spanner import Spanner
from streaming_amd.writer import MDSWriter

__version__ = '0.1.0'

__all__ = [
    'Array', 'BatchDecoder', 'DecodedBatch', 'DeviceBatch', 'FileInfo', 'JointReader',
    'LocalDataset', 'MDSReader', 'MDSWriter', 'Plan', 'RaggedColumn', 'Reader', 'Spanner',
    'decode_batch', 'reader_from_json', 'shard_assignment', 'stage_shards'
]
