"""Repository hygiene checks that need no GPU.

* No module under tests/ defines the same test name twice: a second ``def test_x`` silently
  replaces the first, whose case then stops running (round-5 verdict, weak item 8:
  ``test_groupnorm_large_mean`` was shadowed this way).
"""
import ast
from pathlib import Path

import pytest

TESTS = Path(__file__).resolve().parent


def _duplicates(tree: ast.Module):
    """(scope, name, first line, second line) for every name bound twice by a def / class in one scope."""
    out = []

    def scan(body, scope):
        seen = {}
        for node in body:
            if isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
                if node.name in seen:
                    out.append((scope, node.name, seen[node.name], node.lineno))
                seen[node.name] = node.lineno
                if isinstance(node, ast.ClassDef):
                    scan(node.body, f"{scope}.{node.name}")
    scan(tree.body, "<module>")
    return out


@pytest.mark.parametrize("path", sorted(TESTS.glob("test_*.py")), ids=lambda p: p.name)
def test_no_duplicate_test_names(path):
    dups = _duplicates(ast.parse(path.read_text(), filename=str(path)))
    assert not dups, f"{path.name}: names defined twice (the later one shadows the earlier): {dups}"


def test_duplicate_checker_catches_shadowing():
    src = "def test_a():\n    pass\n\ndef test_b():\n    pass\n\ndef test_a(x):\n    pass\n"
    assert _duplicates(ast.parse(src)) == [("<module>", "test_a", 1, 7)]


def test_production_library_reads_no_environment():
    """include/c2d.h: the library reads no environment variable -- its tuning constants are
    compile-time (csrc/common.h) and A/B candidates are variant builds.  The built libc2d_hip.so
    imports no getenv and holds no C2D_* variable name."""
    import subprocess
    from clap2diffusion_amd import _lib
    so = _lib.LIB_PATH
    if not so.exists():
        pytest.skip("libc2d_hip.so not built")
    und = subprocess.run(["nm", "-D", "--undefined-only", str(so)], capture_output=True, text=True, check=True).stdout
    assert not any(ln.split()[-1].startswith(("getenv", "secure_getenv")) for ln in und.splitlines() if ln.strip())
    assert b"C2D_" not in so.read_bytes()
