"""infinicache_amd — MI355X-native Reed-Solomon erasure coding for the
InfiniCache client (drop-in for reedsolomon.Encoder under
/root/reference/client/ec.go).  See DESIGN.md."""
from .ec import (ALL_DEVICES, DummyEncoder, ErrInvalidInput, ErrInvShardNum, ErrMaxShardNum,  # noqa: F401
                 ErrNotImplemented, ErrReconstructRequired, ErrShardNoData, ErrShardSize,
                 ErrShortData, ErrSingular, ErrTooFewShards, HipError, InvalidArgument, New,
                 NewEncoder, NoDevice, RSEncoder, RSError, device_count, device_ok, host_alloc,
                 host_register, host_unregister, retired_stats, set_slab_bytes, shardmajor_layout)

__all__ = [
    "New", "NewEncoder", "RSEncoder", "DummyEncoder", "RSError", "device_count", "device_ok",
    "ErrInvShardNum", "ErrMaxShardNum", "ErrTooFewShards", "ErrShardNoData", "ErrShardSize",
    "ErrSingular", "ErrShortData", "ErrReconstructRequired", "ErrInvalidInput",
    "ErrNotImplemented", "InvalidArgument", "NoDevice", "HipError", "host_alloc",
    "host_register", "host_unregister", "shardmajor_layout", "ALL_DEVICES", "retired_stats",
    "set_slab_bytes",
]
