"""The tree passes the repository lint (scripts/lint.py: the ruff F401/F811 and
clang-format/doxygen subset that runs without those tools; reference
.github/workflows/lint.yml:13-42)."""

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_tree_is_lint_clean():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "lint.py")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-4000:]


def test_lint_catches_findings(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import lint
    py = tmp_path / "bad.py"
    py.write_text("import os\nx = 1 \n")
    h = tmp_path / "bad.h"
    h.write_text('#include <cuda_runtime.h>\n__global__ void k() {}\nextern "C" int f();\n')
    found = "\n".join(lint.lint([str(py), str(h)]))
    assert "unused import 'os'" in found
    assert "trailing whitespace" in found
    assert "#pragma once" in found
    assert "compatibility-layer marker" in found
    assert "undocumented kernel" in found and "undocumented entry point" in found
