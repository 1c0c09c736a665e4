"""In-tree native build: compiles every HIP/C++ source under ``csrc/`` for gfx950 and links
``tensorflow_distributed_amd/_C.so`` (torch custom ops + native runtime).

No hipify, no torch.utils.cpp_extension JIT cache: kernels are plain HIP C++ (``csrc/kernels/*.hip``)
compiled by ``hipcc --offload-arch=gfx950``; the torch-op binding layer (``csrc/bindings/*.cpp``) is
host-only C++ compiled by g++ against torch's headers. The link step produces one shared object
that travels to the GPU box with the repo snapshot (it is git-ignored, not gpurun-ignored).

Usage:  python -m tensorflow_distributed_amd._build [--force] [-j N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
PKG = os.path.join(ROOT, "tensorflow_distributed_amd")
# Variant builds for A/B kernel experiments: TFD_VARIANT=name + TFD_EXTRA_FLAGS="-DX=1 ..." build
# into build/native-<name>/ and link tensorflow_distributed_amd/_C_<name>.so; load it with
# TFD_NATIVE_LIB=<path>.
VARIANT = os.environ.get("TFD_VARIANT", "")
EXTRA_FLAGS = os.environ.get("TFD_EXTRA_FLAGS", "").split()
HIP_EXTRA_FLAGS = os.environ.get("TFD_HIP_FLAGS", "").split()  # device-compiler-only flags
BUILD = os.path.join(ROOT, "build", "native" + (f"-{VARIANT}" if VARIANT else ""))
OUT = os.path.join(PKG, f"_C_{VARIANT}.so" if VARIANT else "_C.so")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("TFD_OFFLOAD_ARCH", "gfx950")


def _torch_dirs():
    import torch  # noqa: F401  (only for paths)
    tdir = os.path.dirname(torch.__file__)
    return (
        [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")],
        os.path.join(tdir, "lib"),
        bool(torch._C._GLIBCXX_USE_CXX11_ABI),
    )


def _headers():
    return glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)


def _needs(src, obj, hdr_mtime):
    if not os.path.exists(obj):
        return True
    m = os.path.getmtime(obj)
    return os.path.getmtime(src) > m or hdr_mtime > m


def _compile(cmd, src):
    t = subprocess.run(cmd, capture_output=True, text=True)
    if t.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{t.stdout}\n{t.stderr}")
    return src


def build(force: bool = False, jobs: int | None = None, verbose: bool = False) -> str:
    incs, tlib, abi = _torch_dirs()
    os.makedirs(BUILD, exist_ok=True)
    hip_srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")) + glob.glob(os.path.join(CSRC, "comm", "*.hip")))
    cpp_srcs = sorted(glob.glob(os.path.join(CSRC, "bindings", "*.cpp")) + glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    hdr_mtime = max([os.path.getmtime(h) for h in _headers()] + [0])
    common = ["-O3", "-fPIC", "-std=c++17", f"-D_GLIBCXX_USE_CXX11_ABI={int(abi)}", "-I", CSRC] + EXTRA_FLAGS
    hip_flags = common + [
        "-x", "hip", f"--offload-arch={ARCH}", "-D__HIP_PLATFORM_AMD__=1",
        "-ffp-contract=fast", "-munsafe-fp-atomics", "-Wno-unused-result",
        # No packed-fp32 VALU ops (v_pk_fma/mul/add_f32): with them, the SLP-vectorised VALU
        # kernels (conv1, head, wgrad) gave sporadically different results for the same inputs
        # when several processes shared the GPU; without them every stage is bit-reproducible
        # (tools/debug/determinism.py, docs/DESIGN.md section 6). TFD_PACKED_FP32=1 (variant
        # builds only) keeps them for that experiment.
    ] + ([] if os.environ.get("TFD_PACKED_FP32") == "1" else
         ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]) + HIP_EXTRA_FLAGS
    cpp_flags = common + [
        "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-I", os.path.join(ROCM, "include"),
    ] + sum([["-I", i] for i in incs], []) + ["-Wno-deprecated-declarations"]
    # a flag change (build options, torch headers) invalidates every object of this variant
    stamp = os.path.join(BUILD, "flags.stamp")
    sig = repr((hip_flags, cpp_flags))
    if not os.path.exists(stamp) or open(stamp).read() != sig:
        force = True
    jobs_list = []
    objs = []
    for s in hip_srcs:
        o = os.path.join(BUILD, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _needs(s, o, hdr_mtime):
            jobs_list.append(([os.path.join(ROCM, "bin", "hipcc")] + hip_flags + ["-c", s, "-o", o], s))
    for s in cpp_srcs:
        o = os.path.join(BUILD, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _needs(s, o, hdr_mtime):
            jobs_list.append((["g++"] + cpp_flags + ["-c", s, "-o", o], s))
    jobs = jobs or min(8, os.cpu_count() or 4)
    if jobs_list:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            futs = [ex.submit(_compile, c, s) for c, s in jobs_list]
            for f in cf.as_completed(futs):
                s = f.result()
                if verbose:
                    print("compiled", os.path.relpath(s, ROOT), flush=True)
    with open(stamp, "w") as f:
        f.write(sig)
    newest = max([os.path.getmtime(o) for o in objs] + [0])
    if force or jobs_list or not os.path.exists(OUT) or os.path.getmtime(OUT) < newest:
        link = [os.path.join(ROCM, "bin", "hipcc"), "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", OUT] + objs + [
            "-L", tlib, "-Wl,-rpath," + tlib, "-lc10", "-lc10_hip", "-ltorch_cpu", "-ltorch_hip", "-ltorch", "-lrccl",
            "-L", os.path.join(ROCM, "lib"), "-lamdhip64",
        ]
        t = subprocess.run(link, capture_output=True, text=True)
        if t.returncode != 0:
            raise RuntimeError(f"link failed\n{' '.join(link)}\n{t.stdout}\n{t.stderr}")
        if verbose:
            print("linked", os.path.relpath(OUT, ROOT), flush=True)
    return OUT


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    a = ap.parse_args(argv)
    print(build(force=a.force, jobs=a.jobs, verbose=True))


if __name__ == "__main__":
    sys.exit(main())
