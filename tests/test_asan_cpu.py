"""AddressSanitizer run of the library's host code (SURVEY.md §5 sanitizers row): the
HIP sources compiled with -fsanitize=address on the host side (-Xarch_host; nothing is
launched) and linked into tests/asan/abi_host_check.cpp, which sweeps the GEMM planner /
workspace queries over the model shapes and a random sweep and drives every validation path
of the compute entry points.  Any heap / stack error aborts the binary."""
import os
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# the library's compile units as clap2diffusion_amd/build.py compiles them (igemm.hip in its
# four kernel-family parts, runtime.hip with the tuning / plan-override / per-device state)
from clap2diffusion_amd.build import UNITS as _BUILD_UNITS  # noqa: E402

UNITS = [(src, " ".join(f"-D{d}" for d in defs) or None, stem) for src, defs, stem in _BUILD_UNITS]
# ASAN on the host side only (-Xarch_host before each -fsanitize=); device code builds as usual
FLAGS = ["--offload-arch=gfx950", "-O1", "-g", "-Xarch_host", "-fsanitize=address", "-Xarch_host",
         "-fno-omit-frame-pointer", "-std=c++17", "-I", str(ROOT / "include"),
         "-I", str(ROOT / "clap2diffusion_amd" / "csrc")]


@pytest.mark.timeout(600)
def test_abi_host_code_under_asan(tmp_path):
    if not Path(HIPCC).exists():
        pytest.skip("hipcc not available")
    objs = []
    procs = []
    for src, define, stem in UNITS:
        obj = tmp_path / (stem + ".o")
        procs.append(subprocess.Popen([HIPCC, *FLAGS, *([define] if define else []), "-fPIC", "-c",
                                       str(ROOT / "clap2diffusion_amd" / "csrc" / src), "-o", str(obj)],
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
        objs.append(obj)
    for p in procs:
        out, err = p.communicate()
        assert p.returncode == 0, err[-2000:]
    exe = tmp_path / "abi_host_check"
    clang = str(Path(HIPCC).resolve().parent.parent / "lib" / "llvm" / "bin" / "clang++")
    drv = tmp_path / "abi_host_check.o"
    r = subprocess.run([clang, "-O1", "-g", "-fsanitize=address", "-fno-omit-frame-pointer", "-std=c++17",
                        "-I", str(ROOT / "include"), "-c", str(ROOT / "tests" / "asan" / "abi_host_check.cpp"),
                        "-o", str(drv)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    rocm_lib = str(Path(HIPCC).resolve().parent.parent / "lib")
    r = subprocess.run([clang, "-fsanitize=address", str(drv), *map(str, objs), "-L", rocm_lib, "-lamdhip64",
                        f"-Wl,-rpath,{rocm_lib}", "-o", str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and "abi_host_check: ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
