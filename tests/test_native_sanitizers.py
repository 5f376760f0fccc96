"""Host-code sanitizers (SURVEY.md §5 'race detection / sanitizers'): the native runtime core
(csrc/runtime/runtime_core.h — KV block allocator, scheduler, UTF-8 edit distance) is compiled into a
randomised self-test with AddressSanitizer + UndefinedBehaviorSanitizer (and, separately, with the
libstdc++ debug-mode bounds checks) and run on the CPU.  GPU sanitizers / XNACK are
not available on the MI355X pool, so device code is covered by the numerics tests instead."""
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
