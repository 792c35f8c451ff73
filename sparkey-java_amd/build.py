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
OBJ_DIR = os.path.join(HERE, "build", "obj")
SOURCES = [os.path.join(HERE, "csrc", f) for f in (
    "build_kernels.hip", "fused_kernels.hip", "frame3_kernels.hip", "exact_kernels.hip", "shard_kernels.hip",
    "shard_exact_kernels.hip", "lookup_kernels.hip", "append_kernels.hip", "snappy_kernels.hip", "zstd_kernels.hip",
    "sparkey_gpu.cpp", "file_build.cpp", "shard_host.cpp", "knobs.cpp")]
HEADERS = [os.path.join(HERE, "csrc", f) for f in (
    "snappy.hpp", "frame_common.hpp", "build_kernels.hpp", "device_common.hpp", "kernel_utils.hpp", "scan.hpp",
    "place_common.hpp", "lookup.hpp", "append.hpp", "shard_host.hpp", "knobs.hpp")] + [
    os.path.join(ROOT, "include", "sparkey_gpu.h")]
ARCH = os.environ.get("SPARKEY_GPU_ARCH", "gfx950")


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src, obj, verbose):
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-I", os.path.join(ROOT, "include"),
           "-c", "-x", "hip", src, "-o", obj + ".tmp"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(obj + ".tmp", obj)


def build(force: bool = False, verbose: bool = False) -> str:
    """One object per source (compiled in parallel, each only when it or a header changed), then one
    link.  No -fgpu-rdc: every kernel is launched from its own translation unit."""
    from concurrent.futures import ThreadPoolExecutor
    os.makedirs(OBJ_DIR, exist_ok=True)
    os.makedirs(LIB_DIR, exist_ok=True)  # lib/ holds only built files, so a fresh checkout lacks it
    jobs = []
    for s in SOURCES:
        obj = os.path.join(OBJ_DIR, os.path.basename(s) + ".o")
        if force or _stale(obj, [s] + HEADERS + [__file__]):
            jobs.append((s, obj))
    if jobs:
        workers = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", "0")) or (os.cpu_count() or 4)))
        with ThreadPoolExecutor(workers) as ex:
            for f in [ex.submit(_compile, s, o, verbose) for s, o in jobs]:
                f.result()
    objs = [os.path.join(OBJ_DIR, os.path.basename(s) + ".o") for s in SOURCES]
    if force or jobs or _stale(LIB, objs):
        cmd = ["hipcc", f"--offload-arch={ARCH}", "-fPIC", "-shared", "-Wl,--no-undefined"] + objs + ["-o", LIB + ".tmp"]
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
