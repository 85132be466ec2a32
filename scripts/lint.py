#!/usr/bin/env python3
"""Self-contained lint of the repository (no ruff / clang-format / doxygen in
this image; the reference's lint job, .github/workflows/lint.yml:13-42, runs
those three).  The same rules are written down for the real tools in
``ruff.toml`` and ``.clang-format``; this script enforces the subset that can
be checked without them, so CI and ``tests/test_lint.py`` fail on:

Python (``*.py``)
  * syntax errors (``compile``);
  * unused imports (module scope and function scope; ``__init__.py``
    re-exports, ``__future__`` and ``# noqa`` lines excepted) -- ruff F401;
  * duplicate top-level definitions -- ruff F811;
  * lines over 120 columns, tabs, trailing whitespace, missing final newline.
C++ / HIP (``*.h *.hip *.cpp``)
  * headers start with ``#pragma once`` (after the leading comment);
  * no CUDA / hipify / dual-platform markers (``__CUDACC__``,
    ``__HIP_PLATFORM_AMD__``, ``cuda_runtime``, ``hipify``);
  * every ``extern "C"`` entry point and every ``__global__`` kernel has a
    comment in the lines above it (the doxygen job's "documented" check);
  * lines over 120 columns, tabs, trailing whitespace, missing final newline.

usage: python scripts/lint.py [paths...]   (default: the whole tree)
exit status 1 and one ``path:line: message`` per finding when anything fails.
"""

from __future__ import annotations

import ast
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SKIP_DIRS = {".git", "__pycache__", "gpurun_out", "build", ".pytest_cache", "profiles"}
PY_COLS, CXX_COLS = 120, 120
BANNED_CXX = ("__CUDACC__", "__HIP_PLATFORM_AMD__", "__HIP_PLATFORM_NVIDIA__", "cuda_runtime",
              "hipify", "#include <cuda")


def _files(paths):
    for p in paths:
        if os.path.isfile(p):
            yield p
            continue
        for d, dirs, fs in os.walk(p):
            dirs[:] = sorted(x for x in dirs if x not in SKIP_DIRS)
            for f in sorted(fs):
                if f.endswith((".py", ".h", ".hip", ".cpp")):
                    yield os.path.join(d, f)


def _text_checks(path, lines, cols, out):
    for i, ln in enumerate(lines, 1):
        body = ln.rstrip("\n")
        if "\t" in body:
            out.append(f"{path}:{i}: tab character")
        if body != body.rstrip():
            out.append(f"{path}:{i}: trailing whitespace")
        if len(body) > cols and "http" not in body:
            out.append(f"{path}:{i}: line longer than {cols} columns ({len(body)})")
    if lines and not lines[-1].endswith("\n"):
        out.append(f"{path}:{len(lines)}: no newline at end of file")


class _Names(ast.NodeVisitor):
    """Every identifier read anywhere in the module (incl. attribute roots,
    string annotations and __all__ entries)."""

    def __init__(self):
        self.used: set[str] = set()

    def visit_Name(self, node):
        self.used.add(node.id)

    def visit_Attribute(self, node):
        self.generic_visit(node)

    def visit_Constant(self, node):
        if isinstance(node.value, str) and node.value.isidentifier():
            self.used.add(node.value)  # __all__ entries, string annotations
        elif isinstance(node.value, str):
            for tok in re.findall(r"[A-Za-z_][A-Za-z0-9_]*", node.value):
                self.used.add(tok)


def _py_checks(path, src, lines, out):
    try:
        tree = ast.parse(src, path)
    except SyntaxError as e:
        out.append(f"{path}:{e.lineno}: syntax error: {e.msg}")
        return
    names = _Names()
    names.visit(tree)
    is_init = os.path.basename(path) == "__init__.py"
    for node in ast.walk(tree):
        if not isinstance(node, (ast.Import, ast.ImportFrom)):
            continue
        if isinstance(node, ast.ImportFrom) and node.module == "__future__":
            continue
        if "noqa" in lines[node.lineno - 1] or is_init:
            continue
        for a in node.names:
            if a.name == "*":
                continue
            bound = a.asname or a.name.split(".")[0]
            if bound not in names.used:
                out.append(f"{path}:{node.lineno}: unused import {bound!r}")
    seen: dict[str, int] = {}
    for node in tree.body:
        if isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            if node.name in seen and "noqa" not in lines[node.lineno - 1]:
                out.append(f"{path}:{node.lineno}: redefinition of {node.name!r} "
                           f"(first at line {seen[node.name]})")
            seen[node.name] = node.lineno


def _cxx_checks(path, lines, out):
    if path.endswith(".h"):
        code = [ln.strip() for ln in lines if ln.strip() and not ln.strip().startswith("//")]
        if not code or code[0] != "#pragma once":
            out.append(f"{path}:1: header does not start with #pragma once")
    for i, ln in enumerate(lines, 1):
        for b in BANNED_CXX:
            if b in ln:
                out.append(f"{path}:{i}: compatibility-layer marker {b!r}")
    for i, ln in enumerate(lines, 1):
        s = ln.strip()
        entry = s.startswith('extern "C"') and not s.startswith('extern "C" {')
        kernel = s.startswith("__global__") or (s.startswith("template") and i < len(lines)
                                               and lines[i].strip().startswith("__global__"))
        if not (entry or kernel) or ln.rstrip().endswith("\\"):
            continue
        if kernel and s.startswith("__global__") and i >= 2 and \
                lines[i - 2].strip().startswith("template"):
            continue  # documented at its template line
        j = i - 2
        while j >= 0 and (lines[j].strip() == "" or lines[j].strip().startswith("template")):
            j -= 1
        prev = lines[j].strip() if j >= 0 else ""
        if not (prev.startswith("//") or prev.endswith("*/") or prev.startswith("*")):
            out.append(f"{path}:{i}: undocumented {'entry point' if entry else 'kernel'}")


def lint(paths) -> list[str]:
    out: list[str] = []
    for f in _files(paths):
        with open(f, encoding="utf-8") as fh:
            src = fh.read()
        lines = src.splitlines(keepends=True)
        rel = os.path.relpath(f, ROOT)
        if f.endswith(".py"):
            _text_checks(rel, lines, PY_COLS, out)
            _py_checks(rel, src, lines, out)
        else:
            _text_checks(rel, lines, CXX_COLS, out)
            _cxx_checks(rel, lines, out)
    return out


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    paths = argv or [os.path.join(ROOT, p) for p in
                     ("benchmark_dolfinx_amd", "tests", "scripts", "bench.py", "__graft_entry__.py")]
    found = lint(paths)
    for m in found:
        print(m)
    print(f"lint: {len(found)} finding(s)", file=sys.stderr)
    return 1 if found else 0


if __name__ == "__main__":
    raise SystemExit(main())
