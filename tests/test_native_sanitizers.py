"""Host-code sanitizers (SURVEY.md §5 'race detection / sanitizers'): the native runtime core
(csrc/runtime/runtime_core.h — KV block allocator, scheduler, UTF-8 edit distance) is compiled into a
randomised self-test with AddressSanitizer + UndefinedBehaviorSanitizer (and, separately, with the
libstdc++ debug-mode bounds checks) and run on the CPU; so is the argument validation of the torch bindings
(csrc/bindings.cpp, which checks every operand before a kernel launch) against stub launchers.  GPU
sanitizers / XNACK are not available on the MI355X pool, so device code is covered by the numerics tests."""
import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
SRC = ROOT / "csrc" / "tests" / "runtime_selftest.cpp"


@pytest.mark.parametrize("flags", [
    ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"],
    ["-D_GLIBCXX_ASSERTIONS", "-D_GLIBCXX_DEBUG"],
], ids=["asan_ubsan", "glibcxx_debug"])
def test_runtime_core_under_sanitizers(tmp_path, flags):
    if shutil.which("g++") is None:
        pytest.skip("no host compiler")
    exe = tmp_path / "selftest"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", *flags, str(SRC), "-o", str(exe)], check=True,
                   capture_output=True, text=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300,
                       env={"ASAN_OPTIONS": "detect_leaks=1:abort_on_error=0", "UBSAN_OPTIONS": "print_stacktrace=1"})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "runtime selftest ok" in r.stdout


def test_allocator_rejects_double_free_native_and_fallback():
    from llm_based_apache_spark_optimization_amd.runtime import native

    impls = [native._PyBlockAllocator]
    if native.NATIVE:
        impls.append(native._mod.BlockAllocator)
    for cls in impls:
        a = cls(9, 64)
        assert a.alloc(0) == [] and a.num_free == 8
        b = a.alloc(3)
        a.release(b)
        with pytest.raises((ValueError, RuntimeError)):
            a.release(b)  # already free
        c = a.alloc(2)
        with pytest.raises((ValueError, RuntimeError)):
            a.release([c[0], c[0]])  # listed twice: nothing released
        assert a.num_free == 6
        a.release(c)
        assert a.num_free == 8


def test_bindings_validation_under_sanitizers(tmp_path):
    """csrc/tests/bindings_selftest.cpp: every binding's validation accepts well-formed operands (reaching its
    launcher exactly once) and rejects malformed ones before any launch, under ASan + UBSan."""
    if shutil.which("g++") is None or shutil.which("gcc") is None:
        pytest.skip("no host compiler")
    import sysconfig

    from torch.utils import cpp_extension as ce

    names = sorted(set(re.findall(r"\b(lsa_[a-z0-9_]+)\(", (ROOT / "csrc" / "bindings.cpp").read_text())))
    stubs = tmp_path / "stubs.c"
    # launch stubs count calls; the knob setters (no launch) do not
    stubs.write_text("int lsa_stub_calls = 0;\n" + "".join(
        f"int {n}() {{ {'' if 'knobs' in n else '++lsa_stub_calls; '}return 0; }}\n" for n in names))
    san = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer"]
    so = tmp_path / "stubs.o"
    subprocess.run(["gcc", "-c", "-O1", "-g", *san, str(stubs), "-o", str(so)], check=True, capture_output=True, text=True)
    import torch

    inc = [f"-I{p}" for p in ce.include_paths()] + ["-I/opt/rocm/include", f"-I{sysconfig.get_paths()['include']}"]
    lib = ce.library_paths()[0]
    exe = tmp_path / "bindings_selftest"
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-g", *san, "-D__HIP_PLATFORM_AMD__=1",
                        f"-D_GLIBCXX_USE_CXX11_ABI={int(torch._C._GLIBCXX_USE_CXX11_ABI)}", *inc,
                        str(ROOT / "csrc" / "tests" / "bindings_selftest.cpp"), str(so), "-o", str(exe),
                        f"-L{lib}", f"-Wl,-rpath,{lib}", "-lc10", "-ltorch_cpu"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300,
                       env={"ASAN_OPTIONS": "detect_leaks=0:abort_on_error=0", "UBSAN_OPTIONS": "print_stacktrace=1"})
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "bindings selftest ok" in r.stdout
