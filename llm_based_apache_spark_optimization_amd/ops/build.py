"""In-tree build of the native extensions (no hipify, no JIT cache outside the repo).

* ``_lsa_hip``     — the gfx950 HIP kernels (``csrc/kernels/*.hip``) + torch bindings
                     (``csrc/bindings.cpp``), compiled with ``hipcc --offload-arch=gfx950``.
* ``_lsa_runtime`` — host-side C++ runtime (``csrc/runtime/*.cpp``): KV-block allocator,
                     continuous-batching scheduler, Levenshtein distance.  pybind11 only.

Objects are cached under ``build/`` keyed by source mtime + flags, so a rebuild after editing one
kernel recompiles one file.  ``python -m llm_based_apache_spark_optimization_amd.ops.build``.
"""
from __future__ import annotations

import hashlib
import shlex
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent.parent
REPO = PKG_DIR.parent
CSRC = REPO / "csrc"
BUILD = REPO / "build"
ARCH = os.environ.get("LSA_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

HIP_EXT = PKG_DIR / "ops" / "_lsa_hip.so"
RT_EXT = PKG_DIR / "runtime" / "_lsa_runtime.so"


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def _stamp(src: Path, flags: list[str], deps: list[Path]) -> str:
    h = hashlib.sha1()
    h.update(" ".join(flags).encode())
    for p in [src, *deps]:
        h.update(p.read_bytes())
    return h.hexdigest()[:16]


def _compile(src: Path, out_dir: Path, cc: str, flags: list[str], deps: list[Path]) -> Path:
    out_dir.mkdir(parents=True, exist_ok=True)
    key = _stamp(src, flags, deps)
    obj = out_dir / f"{src.stem}.{key}.o"
    if not obj.exists():
        for old in out_dir.glob(f"{src.stem}.*.o"):
            old.unlink()
        _run([cc, *flags, "-c", str(src), "-o", str(obj)])
    return obj


def _torch_flags() -> tuple[list[str], list[str]]:
    import torch
    from torch.utils import cpp_extension as ce

    inc = [f"-I{p}" for p in ce.include_paths(device_type="cuda")]
    py_inc = f"-I{sysconfig.get_paths()['include']}"
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cflags = inc + [py_inc, f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1",
                    "-DTORCH_EXTENSION_NAME=_lsa_hip", "-DTORCH_API_INCLUDE_EXTENSION_H"]
    libdir = ce.library_paths(device_type="cuda")[0]
    ldflags = [f"-L{libdir}", f"-Wl,-rpath,{libdir}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
               "-ltorch_hip", "-ltorch_python"]
    return cflags, ldflags


def hip_sources() -> list[Path]:
    """Every source the gfx950 extension is compiled from (kernels, headers, bindings)."""
    kdir = CSRC / "kernels"
    return sorted(kdir.glob("*.hip")) + sorted(kdir.glob("*.h")) + [CSRC / "bindings.cpp"]


def sources_sha() -> str:
    """Content hash of the extension's sources (relative path + bytes, in path order): what a build provenance
    record pins and what ``ops.ext()`` re-checks on load."""
    h = hashlib.sha256()
    for p in hip_sources():
        h.update(str(p.relative_to(REPO)).encode() + b"\0" + p.read_bytes())
    return h.hexdigest()[:16]


PROVENANCE = HIP_EXT.with_suffix(".provenance.json")


def _write_provenance(kflags: list[str]) -> None:
    import json
    import time

    try:
        ver = subprocess.run([HIPCC, "--version"], capture_output=True, text=True).stdout.splitlines()
    except OSError:
        ver = []
    rec = {"sources_sha": sources_sha(), "so_sha256": hashlib.sha256(HIP_EXT.read_bytes()).hexdigest()[:16],
           "arch": ARCH, "kernel_flags": kflags, "hipcc": next((v for v in ver if "version" in v.lower()), ""),
           "built_unix": int(time.time())}
    PROVENANCE.write_text(json.dumps(rec, indent=1))


def build_hip(jobs: int = 8, verbose: bool = False) -> Path:
    kdir = CSRC / "kernels"
    headers = sorted(kdir.glob("*.h"))
    kflags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=fast", "-Wno-unused-result"]
    kflags += shlex.split(os.environ.get("LSA_HIP_EXTRA", ""))  # experiment knobs, e.g. -DLSA_ATTN_NT=0
    srcs = sorted(kdir.glob("*.hip"))
    tflags, ldflags = _torch_flags()
    bflags = ["-O2", "-std=c++17", "-fPIC", "-Wno-deprecated-declarations", "-Wno-unused-result", *tflags]
    odir = BUILD / ARCH
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        futs = [ex.submit(_compile, s, odir, HIPCC, kflags, headers) for s in srcs]
        futs.append(ex.submit(_compile, CSRC / "bindings.cpp", odir, HIPCC, bflags, headers))
        objs = [f.result() for f in futs]
    key = hashlib.sha1("".join(sorted(o.name for o in objs)).encode()).hexdigest()[:16]
    stamp = HIP_EXT.with_suffix(".stamp")
    if HIP_EXT.exists() and stamp.exists() and stamp.read_text() == key:
        if not PROVENANCE.exists():
            _write_provenance(kflags)
        return HIP_EXT
    _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(HIP_EXT), *ldflags])
    stamp.write_text(key)
    _write_provenance(kflags)
    if verbose:
        print(f"built {HIP_EXT}")
    return HIP_EXT


def build_runtime(verbose: bool = False) -> Path:
    import pybind11

    rdir = CSRC / "runtime"
    srcs = sorted(rdir.glob("*.cpp"))
    headers = sorted(rdir.glob("*.h"))
    flags = ["-O3", "-std=c++17", "-fPIC", "-Wall", f"-I{pybind11.get_include()}",
             f"-I{sysconfig.get_paths()['include']}", "-fvisibility=hidden"]
    odir = BUILD / "host"
    with ThreadPoolExecutor(max_workers=4) as ex:
        objs = list(ex.map(lambda s: _compile(s, odir, "g++", flags, headers), srcs))
    key = hashlib.sha1("".join(sorted(o.name for o in objs)).encode()).hexdigest()[:16]
    stamp = RT_EXT.with_suffix(".stamp")
    if RT_EXT.exists() and stamp.exists() and stamp.read_text() == key:
        return RT_EXT
    _run(["g++", "-shared", "-fPIC", *map(str, objs), "-o", str(RT_EXT)])
    stamp.write_text(key)
    if verbose:
        print(f"built {RT_EXT}")
    return RT_EXT


def build_all(verbose: bool = True) -> None:
    build_runtime(verbose=verbose)
    build_hip(jobs=int(os.environ.get("MAX_JOBS", "8")), verbose=verbose)


if __name__ == "__main__":
    build_all(verbose=True)
    sys.exit(0)
