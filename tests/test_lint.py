"""The tree stays clean under tools/lint.py (syntax, unused imports,
whitespace, line length) -- the repository's lint gate (no ruff / flake8 in
the image; .pre-commit-config.yaml runs the same script)."""
from __future__ import annotations

import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_lint_clean():
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'tools', 'lint.py')],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-4000:]
