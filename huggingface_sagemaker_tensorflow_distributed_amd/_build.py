"""In-tree build of the native extension ``_C.so`` (gfx950 only).

Every ``csrc/kernels/*.hip`` is compiled by ``hipcc --offload-arch=gfx950`` into its own object
(kernels never include torch headers, so they compile in seconds), ``csrc/bindings.cpp`` and
``csrc/comm/*.cpp`` are compiled against torch's headers, and everything is linked into
``huggingface_sagemaker_tensorflow_distributed_amd/_C.so`` next to this file — in-tree, so the
``.so`` travels to the GPU box with the repo snapshot. No hipify pass, no CUDA shims: the sources
are HIP.

    python -m huggingface_sagemaker_tensorflow_distributed_amd._build [-v] [--force]
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import json
import os
import subprocess
import sys
import sysconfig

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "hsd")
OUT = os.path.join(PKG_DIR, "_C.so")
# debug variant: -DHSD_DEBUG (synchronising launch checks, device asserts, host-side
# index range checks), separate objects, imported as _C_debug when HSD_DEBUG=1
BUILD_DEBUG = os.path.join(ROOT, "build", "hsd_debug")
OUT_DEBUG = os.path.join(PKG_DIR, "_C_debug.so")
ARCH = os.environ.get("HSD_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

COMMON_FLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wno-unused-result",
                "-Wno-deprecated-declarations", "-Wno-unused-command-line-argument"]


def _torch_flags():
    import torch
    from torch.utils import cpp_extension as ce

    inc = ce.include_paths()
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    py_inc = sysconfig.get_paths()["include"]
    cflags = [f"-I{p}" for p in inc] + [f"-I{py_inc}", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
                                          "-DTORCH_API_INCLUDE_EXTENSION_H",
                                          "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1"]
    libdir = ce.library_paths()[0]
    ldflags = [f"-L{libdir}", f"-Wl,-rpath,{libdir}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
               "-ltorch_hip", "-ltorch_python", "-lamdhip64"]
    rccl = os.path.join(libdir, "librccl.so")
    if os.path.exists(rccl):
        ldflags += [rccl]
    return cflags, ldflags


def _sources():
    kernels = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    hosts = [os.path.join(CSRC, "bindings.cpp")] + sorted(glob.glob(os.path.join(CSRC, "comm", "*.cpp")))
    return kernels, hosts


def _headers():
    return sorted(glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True))


def _digest(path: str, extra: str) -> str:
    h = hashlib.sha1(extra.encode())
    with open(path, "rb") as f:
        h.update(f.read())
    for hd in _headers():
        with open(hd, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _obj_path(src: str, build_dir: str) -> str:
    rel = os.path.relpath(src, CSRC).replace(os.sep, "__")
    return os.path.join(build_dir, rel + ".o")


def _compile(src: str, flags, verbose: bool, build_dir: str = BUILD):
    obj = _obj_path(src, build_dir)
    stamp = obj + ".sha1"
    dig = _digest(src, " ".join(flags))
    if os.path.exists(obj) and os.path.exists(stamp) and open(stamp).read() == dig:
        return obj, False
    cmd = [HIPCC, *flags, "-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
    with open(stamp, "w") as f:
        f.write(dig)
    return obj, True


def build(verbose: bool = False, force: bool = False, jobs: int = 0, debug: bool = False) -> str:
    build_dir, out = (BUILD_DEBUG, OUT_DEBUG) if debug else (BUILD, OUT)
    os.makedirs(build_dir, exist_ok=True)
    if force:
        for f in glob.glob(os.path.join(build_dir, "*")):
            os.remove(f)
    cflags, ldflags = _torch_flags()
    cflags = cflags + ["-DTORCH_EXTENSION_NAME=" + ("_C_debug" if debug else "_C")]
    kernels, hosts = _sources()
    incs = [f"-I{CSRC}", f"-I{os.path.join(CSRC, 'kernels')}"]
    common = COMMON_FLAGS + (["-DHSD_DEBUG=1"] if debug else [])
    jobs = jobs or min(16, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(jobs) as ex:
        futs = [ex.submit(_compile, s, common + incs, verbose, build_dir) for s in kernels]
        futs += [ex.submit(_compile, s, common + incs + cflags, verbose, build_dir) for s in hosts]
        results = [f.result() for f in futs]
    objs = [o for o, _ in results]
    changed = any(c for _, c in results) or not os.path.exists(out)
    manifest = os.path.join(build_dir, "link.json")
    want = json.dumps({"objs": objs, "ld": ldflags})
    if not changed and os.path.exists(manifest) and open(manifest).read() == want:
        return out
    tmp = out + ".tmp"
    cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-fPIC", *objs, "-o", tmp, *ldflags]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, out)
    with open(manifest, "w") as f:
        f.write(want)
    return out


if __name__ == "__main__":
    v = "-v" in sys.argv
    out = build(verbose=v, force="--force" in sys.argv, debug="--debug" in sys.argv)
    print(out)
