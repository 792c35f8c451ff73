"""MI355X-native Sparkey hash-file builder: the com.spotify.sparkey writer API with writeHash() on gfx950.

Importing this package loads libsparkey_gpu.so; there is no CPU fallback.  Batched GPU lookups over a
built hash file: sparkey.reader.GpuHashReader.
"""
from ._native import (BuildStats, Plan, SparkeyGpuError, SparkeyIOError, SparkeyRuntimeError, build_index_file,
                      build_index_mem, index_size, make_opts, version)
from .log_writer import CompressionType, LogHeader, LogWriter, vlq_bytes, vlq_size
from .writer import ConstructionMethod, HashType, Sparkey, SparkeyWriter, renameFile

__all__ = ["Sparkey", "SparkeyWriter", "HashType", "ConstructionMethod", "CompressionType", "LogWriter", "LogHeader",
           "SparkeyIOError", "SparkeyRuntimeError", "SparkeyGpuError", "Plan", "BuildStats", "build_index_file",
           "build_index_mem", "index_size", "make_opts", "version", "renameFile", "vlq_bytes", "vlq_size"]
