"""Host-side mirror of com.spotify.sparkey's writer API (SparkeyWriter / SingleThreadedSparkeyWriter /
Sparkey facade) whose writeHash() builds the .spi on the GPU through the C-ABI.

Names, argument meaning and error behaviour follow the reference:
  SparkeyWriter.java:22-136, SingleThreadedSparkeyWriter.java:25-174, Sparkey.java:41-236,
  Util.renameFile (Util.java:278-315).
"""
from __future__ import annotations

import enum
import os
import random
import uuid

from . import _native
from .log_writer import CompressionType, LogWriter


class HashType(enum.Enum):
    """HashType.java: HASH_64_BITS(8), HASH_32_BITS(4)."""
    HASH_64_BITS = 8
    HASH_32_BITS = 4

    def size(self) -> int:
        return self.value


class ConstructionMethod(enum.IntEnum):
    """SparkeyWriter.ConstructionMethod."""
    AUTO = _native.METHOD_AUTO
    IN_MEMORY = _native.METHOD_IN_MEMORY
    SORTING = _native.METHOD_SORTING


def _free_memory() -> int:
    try:
        return os.sysconf("SC_AVPHYS_PAGES") * os.sysconf("SC_PAGE_SIZE")
    except (ValueError, OSError):
        return 1 << 30


def renameFile(src: str, dest: str) -> None:
    """Util.renameFile (Util.java:278-315): rename with a backup of an existing target and rollback."""
    if not os.path.exists(src):
        raise FileNotFoundError(src)
    if os.path.abspath(src) == os.path.abspath(dest):
        return
    if not os.path.exists(dest):
        os.rename(src, dest)
        return
    backup = os.path.join(os.path.dirname(dest) or ".", os.path.basename(dest) + "-backup" + str(uuid.uuid4()))
    if os.path.exists(backup):
        raise OSError("Expected duplicate temporary backup file: " + backup)
    os.rename(dest, backup)
    try:
        os.rename(src, dest)
        try:
            os.remove(backup)
        except OSError:
            pass
    except OSError as e:
        try:
            os.rename(backup, dest)
        except OSError:
            pass
        raise OSError(f"Could not rename {src} to {dest}") from e


class SparkeyWriter:
    """SingleThreadedSparkeyWriter: not thread-safe, one writer per thread (Sparkey.java:36)."""

    def __init__(self, index_file: str, log_writer: LogWriter, device: int = 0):
        self.indexFile = index_file
        self.logFile = log_writer.path
        self.logWriter = log_writer
        self.sparsity = 0.0
        self.hashType = None
        self.fsync = False
        self.hashSeed = 0
        self.maxMemory = -1
        self.method = ConstructionMethod.AUTO
        self.device = device
        self.lastBuildStats = None

    # --- SparkeyWriter setters (SingleThreadedSparkeyWriter.java:115-143) ---
    def setFsync(self, fsync: bool) -> None:
        self.fsync = bool(fsync)

    def setHashType(self, hash_type) -> None:
        self.hashType = hash_type

    def setHashSparsity(self, sparsity: float) -> None:
        self.sparsity = float(sparsity)

    def setHashSeed(self, seed: int) -> None:
        self.hashSeed = int(seed)

    def setMaxMemory(self, max_memory: int) -> None:
        self.maxMemory = int(max_memory)

    def setConstructionMethod(self, method) -> None:
        self.method = ConstructionMethod(method)

    # --- append path ---
    def put(self, key, value) -> None:
        self.logWriter.put(key, value)

    def delete(self, key) -> None:
        self.logWriter.delete(key)

    def flush(self) -> None:
        self.logWriter.flush(self.fsync)

    def close(self) -> None:
        self.logWriter.close(self.fsync)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # --- the hot path: writeHash (SingleThreadedSparkeyWriter.java:89-108) ---
    def writeHash(self, hash_type=None) -> None:
        if hash_type is not None:
            self.setHashType(hash_type)
        self.flush()
        parent = os.path.dirname(os.path.abspath(self.indexFile))
        tmp = os.path.join(parent, os.path.basename(self.indexFile) + "-tmp" + str(uuid.uuid4()))
        try:
            seed = self.hashSeed
            if seed == 0:
                seed = random.getrandbits(32) - (1 << 31) or 1
            max_memory = self.maxMemory
            if max_memory < 0:
                max_memory = _free_memory() // 2
            opts = _native.make_opts(hash_size=0 if self.hashType is None else HashType(self.hashType).size(),
                                     hash_seed=seed, sparsity=self.sparsity,
                                     max_memory=max(max_memory, 10 * 1024 * 1024), method=int(self.method),
                                     device=self.device)
            self.lastBuildStats = _native.build_index_file(self.logFile, tmp, opts, self.fsync)
            renameFile(tmp, self.indexFile)
        finally:
            if os.path.exists(tmp):
                os.remove(tmp)


class Sparkey:
    """Static facade (Sparkey.java:41-236)."""

    @staticmethod
    def setEnding(file: str, ending: str) -> str:
        if file is None:
            return None
        d, name = os.path.split(file)
        if name.endswith(ending):
            return file
        if name.endswith(".spi") or name.endswith(".spl"):
            return os.path.join(d, name[:name.rindex(".")] + ending)
        if name.endswith("."):
            return os.path.join(d, name[:-1] + ending)
        return os.path.join(d, name + ending)

    @staticmethod
    def getLogFile(file: str) -> str:
        return Sparkey.setEnding(file, ".spl")

    @staticmethod
    def getIndexFile(file: str) -> str:
        return Sparkey.setEnding(file, ".spi")

    @staticmethod
    def createNew(file: str, compressionType=CompressionType.NONE, compressionBlockSize: int = 0,
                  file_identifier=None, device: int = 0) -> SparkeyWriter:
        index_file = Sparkey.getIndexFile(file)
        if os.path.exists(index_file):
            os.remove(index_file)
        log_file = Sparkey.getLogFile(file)
        if os.path.exists(log_file):
            os.remove(log_file)
        lw = LogWriter.createNew(log_file, compressionType, compressionBlockSize, file_identifier)
        return SparkeyWriter(index_file, lw, device)

    @staticmethod
    def append(file: str, device: int = 0) -> SparkeyWriter:
        log_file = Sparkey.getLogFile(file)
        if not os.path.exists(log_file):
            raise FileNotFoundError("File not found: " + log_file)
        return SparkeyWriter(Sparkey.getIndexFile(file), LogWriter.openExisting(log_file), device)

    @staticmethod
    def appendOrCreate(file: str, compressionType=CompressionType.NONE, compressionBlockSize: int = 0,
                       device: int = 0) -> SparkeyWriter:
        log_file = Sparkey.getLogFile(file)
        if os.path.exists(log_file):
            lw = LogWriter.openExisting(log_file)
        else:
            lw = LogWriter.createNew(log_file, compressionType, compressionBlockSize)
        return SparkeyWriter(Sparkey.getIndexFile(file), lw, device)

    @staticmethod
    def writeHash(file: str, hashType=None, device: int = 0) -> None:
        w = Sparkey.append(file, device)
        w.writeHash(hashType)
        w.close()
