"""Build an experiment variant of the gfx950 extension next to the in-tree one: the named kernel sources compiled with
extra flags (objects under build/variants/<name>/), everything else from the in-tree objects, linked into
variants/<name>.so -- load it with LSA_HIP_SO=variants/<name>.so (scripts/ab_build_ttft.sh, ttft_knob_ab.py).
Usage: python scripts/build_variant.py <name> <source.hip,...> <flag> [flag ...]
  e.g. python scripts/build_variant.py mma_dma gemm_tile256.hip -DLSA_SK_MMA_DMA=1"""
import shlex
import os
import sys
from concurrent.futures import ThreadPoolExecutor

sys.path.insert(0, ".")
from llm_based_apache_spark_optimization_amd.ops import build as b  # noqa: E402

name, which, extra = sys.argv[1], set(sys.argv[2].split(",")), sys.argv[3:]
kdir = b.CSRC / "kernels"
headers = sorted(kdir.glob("*.h"))
kflags = [f"--offload-arch={b.ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=fast", "-Wno-unused-result"]
kflags += shlex.split(os.environ.get("LSA_HIP_EXTRA", ""))
tflags, ldflags = b._torch_flags()
bflags = ["-O2", "-std=c++17", "-fPIC", "-Wno-deprecated-declarations", "-Wno-unused-result", *tflags]
vdir = b.BUILD / "variants" / name
with ThreadPoolExecutor(max_workers=8) as ex:
    futs = [ex.submit(b._compile, s, vdir if s.name in which else b.BUILD / b.ARCH, b.HIPCC,
                      kflags + (extra if s.name in which else []), headers) for s in sorted(kdir.glob("*.hip"))]
    futs.append(ex.submit(b._compile, b.CSRC / "bindings.cpp", b.BUILD / b.ARCH, b.HIPCC, bflags, headers))
    objs = [f.result() for f in futs]
out = b.REPO / "variants" / f"{name}.so"
out.parent.mkdir(exist_ok=True)
b._run([b.HIPCC, f"--offload-arch={b.ARCH}", "-shared", "-fPIC", *map(str, objs), "-o", str(out), *ldflags])
print(out)
