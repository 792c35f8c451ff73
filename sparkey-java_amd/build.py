"""Builds libsparkey_gpu.so for gfx950 in-tree (hipcc -shared), plus the JNI shim where a JDK exists.

    python sparkey-java_amd/build.py            # -> sparkey-java_amd/lib/libsparkey_gpu.so
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_DIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIB_DIR, "libsparkey_gpu.so")
SOURCES = [os.path.join(HERE, "csrc", f) for f in ("build_kernels.hip", "fused_kernels.hip", "frame2_kernels.hip", "frame3_kernels.hip", "exact_kernels.hip", "shard_kernels.hip", "shard_exact_kernels.hip",
                                                      "lookup_kernels.hip", "append_kernels.hip", "snappy_kernels.hip", "zstd_kernels.hip", "sparkey_gpu.cpp", "file_build.cpp")]
HEADERS = [os.path.join(HERE, "csrc", f) for f in ("snappy.hpp", "frame_common.hpp", "build_kernels.hpp", "device_common.hpp", "kernel_utils.hpp", "scan.hpp", "place_common.hpp",
                                                      "lookup.hpp", "append.hpp")] + [
    os.path.join(ROOT, "include", "sparkey_gpu.h")]
ARCH = os.environ.get("SPARKEY_GPU_ARCH", "gfx950")


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(LIB_DIR, exist_ok=True)
    if force or _stale(LIB, SOURCES + HEADERS + [__file__]):
        cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wl,--no-undefined", "-Wall",
               "-I", os.path.join(ROOT, "include")]
        for s in SOURCES:
            cmd += ["-x", "hip", s]
        cmd += ["-o", LIB + ".tmp"]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        os.replace(LIB + ".tmp", LIB)
    _build_jni(verbose)
    return LIB


def _build_jni(verbose: bool) -> None:
    """Compiles the JNI shim only where a JDK provides jni.h (never in this image)."""
    java_home = os.environ.get("JAVA_HOME", "")
    jni_h = os.path.join(java_home, "include", "jni.h") if java_home else ""
    if not jni_h or not os.path.exists(jni_h):
        return
    out = os.path.join(LIB_DIR, "libsparkey_gpu_jni.so")
    src = os.path.join(HERE, "jni", "sparkey_gpu_jni.c")
    cmd = ["gcc", "-O2", "-fPIC", "-shared", "-I", os.path.join(java_home, "include"),
           "-I", os.path.join(java_home, "include", "linux"), "-I", os.path.join(ROOT, "include"), src,
           "-L", LIB_DIR, "-lsparkey_gpu", "-Wl,-rpath,$ORIGIN", "-o", out]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
