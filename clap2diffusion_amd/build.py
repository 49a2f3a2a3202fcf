"""Build libc2d_hip.so (gfx950) in-tree with hipcc.

Usage: python -m clap2diffusion_amd.build [--force] [--jobs N]
The shared library lands next to this file so it travels with the repo
snapshot to the GPU box (it is git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
LIB = PKG / "libc2d_hip.so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
SOURCES = ["igemm.hip", "norm.hip", "attention.hip", "elementwise.hip", "audio.hip", "runtime.hip"]
# compile units: igemm.hip once per kernel family (C2D_IGEMM_PART, see its header) so
# the families build in parallel; (source, extra defines, object stem)
UNITS = [("igemm.hip", (f"C2D_IGEMM_PART={k}",), f"igemm_p{k}") for k in range(5)] + \
        [(s, (), Path(s).stem) for s in SOURCES[1:]]
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
         "-Wno-unused-result", "-I", str(ROOT / "include")]
# attention rescales its MFMA accumulators with VALU every tile: keep them in
# arch VGPRs (gfx950 MFMA can write them) instead of AGPRs + accvgpr copies
# (-fno-honor-nans: the softmax max chains fold into v_max3 without canonicalising v_max.
# Scores are finite unless a caller's attention_mask holds -inf (c2d_attention_fwd_mask):
# infinities stay honoured, a row with a finite score is exact and an all -inf row comes
# out NaN as torch's softmax does; tests/test_kernels_gpu.py::test_attention_query_mask)
EXTRA = {"attention.hip": ["-Xarch_device", "-mllvm=-amdgpu-mfma-vgpr-form=true", "-fno-honor-nans"]}


def _digest(defines=()) -> str:
    h = hashlib.sha256()
    h.update(repr((FLAGS, EXTRA, tuple(defines), UNITS)).encode())
    for f in sorted(CSRC.iterdir()):
        if f.suffix in (".hip", ".h", ".cpp"):
            h.update(f.name.encode())
            h.update(f.read_bytes())
    h.update((ROOT / "include" / "c2d.h").read_bytes())
    h.update(" ".join(FLAGS).encode())
    return h.hexdigest()[:16]


def _compile(unit, build_dir: Path, defines=(), flags=()) -> Path:
    src, udefs, stem = unit
    obj = build_dir / (stem + ".o")
    cmd = [HIPCC, *FLAGS, *[f"-D{d}" for d in (*defines, *udefs)], *EXTRA.get(src, []), *flags, "-c", str(CSRC / src),
           "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, jobs: int = 4, verbose: bool = True, ablation: bool = False,
          variant: str = "", variant_defines: tuple = (), variant_flags: tuple = ()) -> Path:
    """ablation=True builds libc2d_hip_abl.so with -DC2D_ENABLE_ABLATION (timing-ablation
    switches live; wrong results by design) for scripts/gpu_abl_tiles.sh via C2D_LIB; the
    production libc2d_hip.so never contains them.  variant="x" with variant_defines builds
    libc2d_hip_x.so (compile-time A/B candidates, loaded through C2D_LIB)."""
    defines = ("C2D_ENABLE_ABLATION",) if ablation else tuple(variant_defines)
    if variant_flags and not variant:
        raise ValueError("extra compiler flags only for a named A/B variant")
    stem = "libc2d_hip_abl" if ablation else (f"libc2d_hip_{variant}" if variant else "libc2d_hip")
    lib_path = PKG / f"{stem}.so"
    stamp = PKG / f".{stem}.stamp"
    dig = _digest(defines + tuple(variant_flags))
    if lib_path.exists() and stamp.exists() and stamp.read_text().strip() == dig and not force:
        if verbose:
            print(f"[c2d] {lib_path.name} up to date ({dig})")
        return lib_path
    build_dir = ROOT / "build" / ("c2d_abl" if ablation else (f"c2d_{variant}" if variant else "c2d"))
    build_dir.mkdir(parents=True, exist_ok=True)
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda u: _compile(u, build_dir, defines, variant_flags), UNITS))
    tmp = lib_path.with_suffix(".so.tmp")
    cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(tmp), *map(str, objs)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    # a kernel whose host stub was silently dropped leaves an undefined c2d:: symbol
    # that only dlopen reports; fail the build instead
    nm = subprocess.run(["nm", "-C", "--undefined-only", str(tmp)], capture_output=True, text=True)
    bad = [ln.strip() for ln in nm.stdout.splitlines() if "c2d::" in ln and ln.split()[0] == "U"]
    if bad:
        tmp.unlink()
        raise RuntimeError("undefined device-kernel stubs in libc2d_hip.so:\n  " + "\n  ".join(bad))
    os.replace(tmp, lib_path)
    stamp.write_text(dig)
    if verbose:
        print(f"[c2d] built {lib_path} ({dig})")
    return lib_path


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=4)
    ap.add_argument("--ablation", action="store_true", help="build libc2d_hip_abl.so (timing ablations)")
    ap.add_argument("--variant", default="", help="build libc2d_hip_<variant>.so with --define D ...")
    ap.add_argument("--define", action="append", default=[])
    ap.add_argument("--cflag", action="append", default=[], help="extra hipcc flag (variant builds only)")
    a = ap.parse_args()
    build(force=a.force, jobs=a.jobs, ablation=a.ablation, variant=a.variant, variant_defines=tuple(a.define),
          variant_flags=tuple(a.cflag))
    sys.exit(0)
