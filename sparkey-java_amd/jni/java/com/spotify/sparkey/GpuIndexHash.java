/*
 * GpuIndexHash.java -- the Java half of the drop-in boundary (INTEGRATION.md §1).
 *
 * Dropped into sparkey-java's own source tree (src/main/java/com/spotify/sparkey/) so that it reaches
 * the package-private types, it replaces IndexHash.createNew (IndexHash.java:131-167) with the MI355X
 * build behind the C-ABI (include/sparkey_gpu.h: sparkey_build_index_file), through the JNI shim
 * sparkey-java_amd/jni/sparkey_gpu_jni.c (libsparkey_gpu_jni.so, linked to libsparkey_gpu.so).  The
 * one caller, SingleThreadedSparkeyWriter.writeHash (SingleThreadedSparkeyWriter.java:89-108), keeps
 * seed and maxMemory resolution, the -tmp<UUID> file and Util.renameFile; only its line 103 changes:
 *
 *     if (GpuIndexHash.enabled()) {
 *       GpuIndexHash.createNew(newFile, logFile, hashType, sparsity, fsync, hashSeed,
 *                              Math.max(maxMemory, 10*1024*1024L), method);
 *     } else {
 *       IndexHash.createNew(newFile, logFile, hashType, sparsity, fsync, hashSeed,
 *                           Math.max(maxMemory, 10*1024*1024L), method);
 *     }
 *
 * Exceptions are the reference's (the shim's throw_for): IOException for LogHeader.read, "No free
 * slots in the hash" and file I/O; RuntimeException for "Corrupt data" / "Invalid data - reference to
 * delete entry", "Too long VLQ value", records the log iterator cannot read, and device failures;
 * IllegalArgumentException for bad options.
 *
 * No JDK exists in the image this repository is built in: this file is compiled by a maintainer's
 * Maven build, and tests/test_jni_shim.py checks that its native method matches the shim's JNI symbol
 * and signature.
 */
package com.spotify.sparkey;

import java.io.File;
import java.io.IOException;

/** MI355X hash-file build; same contract as {@link IndexHash#createNew}. */
final class GpuIndexHash {
  /** -Dsparkey.gpu=true routes writeHash through the GPU build. */
  private static final boolean ENABLED = Boolean.getBoolean("sparkey.gpu");
  /** First device of the build (-Dsparkey.gpu.device, default 0). */
  private static final int DEVICE = Integer.getInteger("sparkey.gpu.device", 0);
  /** Devices the log's byte range is sharded over (-Dsparkey.gpu.count; 1: one GPU). */
  private static final int NUM_GPUS = Integer.getInteger("sparkey.gpu.count", 1);

  static {
    if (ENABLED) {
      System.loadLibrary("sparkey_gpu_jni");  // links libsparkey_gpu.so
    }
  }

  private GpuIndexHash() {}

  static boolean enabled() {
    return ENABLED;
  }

  /**
   * IndexHash.createNew (IndexHash.java:131-167) on the GPU: the same arguments, the same .spi bytes
   * at indexFile, the same exceptions.
   */
  static void createNew(File indexFile, File logFile, HashType hashType, double sparsity, boolean fsync,
                        int hashSeed, long maxMemory, SparkeyWriter.ConstructionMethod method)
      throws IOException {
    // hashType == null: auto (32-bit below 2^23 PUTs, IndexHash.java:141-143); else its byte size
    int hashSize = hashType == null ? 0 : hashType.size();
    createNew0(indexFile.getPath(), logFile.getPath(), hashSize, sparsity, fsync, hashSeed, maxMemory,
               method.ordinal(), DEVICE, NUM_GPUS, null);
  }

  /**
   * Java_com_spotify_sparkey_GpuIndexHash_createNew0 (sparkey_gpu_jni.c).  method: the ordinal of
   * SparkeyWriter.ConstructionMethod (AUTO, IN_MEMORY, SORTING); statsOut, when not null, receives
   * the build's statistics (sparkey_build_stats, in declaration order).
   */
  private static native void createNew0(String indexFile, String logFile, int hashSize, double sparsity,
                                        boolean fsync, int hashSeed, long maxMemory, int method, int device,
                                        int numGpus, long[] statsOut) throws IOException;
}
