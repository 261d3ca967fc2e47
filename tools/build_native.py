#!/usr/bin/env python3
"""Build the native libraries in-tree.

* ``libdtm_kernels.so`` - every HIP kernel in ``csrc/kernels/*.hip`` compiled for gfx950 with
  hipcc (C ABI, called through ctypes from ``distributed_tensorflow_models_amd.ops``).
* ``libdtm_runtime.so`` - the host C++ runtime in ``csrc/runtime/*.cpp`` (TensorBundle
  checkpoint reader/writer, crc32c, CIFAR-binary / TFRecord readers, staleness clock).

Incremental: an object is rebuilt only when its source or a header is newer.
Usage: python tools/build_native.py [--force] [-j N] [--debug-asan]
"""
import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT_DIR = os.path.join(ROOT, "distributed_tensorflow_models_amd", "_native")
OBJ_DIR = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")


def _newer(src_list, target):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in src_list)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("command failed: %s\n%s" % (" ".join(cmd), r.stdout))
    return r.stdout


def build(force=False, jobs=None, asan=False, verbose=False):
    os.makedirs(OUT_DIR, exist_ok=True)
    os.makedirs(OBJ_DIR, exist_ok=True)
    jobs = jobs or min(8, os.cpu_count() or 4)
    kdir = os.path.join(ROOT, "csrc", "kernels")
    rdir = os.path.join(ROOT, "csrc", "runtime")
    kheaders = glob.glob(os.path.join(kdir, "*.h"))
    rheaders = glob.glob(os.path.join(rdir, "*.h"))
    hip_srcs = sorted(glob.glob(os.path.join(kdir, "*.hip")))
    cpp_srcs = sorted(glob.glob(os.path.join(rdir, "*.cpp")))

    jobs_list = []
    hip_objs = []
    for s in hip_srcs:
        o = os.path.join(OBJ_DIR, os.path.basename(s) + ".o")
        hip_objs.append(o)
        if force or _newer([s] + kheaders, o):
            jobs_list.append([HIPCC, "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC",
                              "-munsafe-fp-atomics", "-c", s, "-o", o])
    cpu_objs = []
    for s in cpp_srcs:
        o = os.path.join(OBJ_DIR, os.path.basename(s) + ".o")
        cpu_objs.append(o)
        if force or _newer([s] + rheaders, o):
            flags = ["-O2", "-std=c++17", "-fPIC", "-Wall", "-pthread"]
            if asan:
                flags = ["-O1", "-g", "-std=c++17", "-fPIC", "-pthread", "-fsanitize=address,undefined",
                         "-fno-omit-frame-pointer"]
            jobs_list.append([CXX] + flags + ["-c", s, "-o", o])
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for out in ex.map(_run, jobs_list):
            if verbose and out.strip():
                print(out)
    klib = os.path.join(OUT_DIR, "libdtm_kernels.so")
    if hip_objs and (force or _newer(hip_objs, klib)):
        _run([HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", klib] + hip_objs)
    rlib = os.path.join(OUT_DIR, "libdtm_runtime.so")
    if cpu_objs and (force or _newer(cpu_objs, rlib)):
        extra = ["-fsanitize=address,undefined"] if asan else []
        _run([CXX, "-shared", "-fPIC", "-pthread", "-o", rlib] + cpu_objs + extra)
    return klib, rlib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--debug-asan", action="store_true", help="host runtime with ASan/UBSan")
    ap.add_argument("-v", action="store_true")
    a = ap.parse_args()
    k, r = build(a.force, a.j, a.debug_asan, a.v)
    print("built", k, r)


if __name__ == "__main__":
    sys.exit(main())
