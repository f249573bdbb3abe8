"""Dependency-free lint for the repository (no ruff / flake8 in the image).

Checks every tracked Python file for: syntax errors, imported names that are
never used (``__init__.py`` re-exports and ``# noqa`` lines excepted),
tabs, trailing whitespace and lines longer than ``MAX_LINE``; and every HIP /
C++ source for tabs and trailing whitespace.  Exit status 1 on findings.

    python tools/lint.py [paths...]
"""
from __future__ import annotations

import ast
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAX_LINE = 120
PY_DIRS = ('distributed_kfac_pytorch_amd', 'examples', 'tests', 'tools', 'scripts')
PY_FILES = ('bench.py', 'setup.py', '__graft_entry__.py')
NATIVE_DIRS = ('csrc',)


def _unused_imports(tree: ast.AST, lines: list[str]) -> list[tuple[int, str]]:
    imported: dict[str, int] = {}
    for node in ast.walk(tree):
        if isinstance(node, (ast.Import, ast.ImportFrom)):
            if isinstance(node, ast.ImportFrom) and node.module == '__future__':
                continue
            for a in node.names:
                name = (a.asname or a.name).split('.')[0]
                if a.name == '*':
                    continue
                imported[name] = node.lineno
    used: set[str] = set()
    for node in ast.walk(tree):
        if isinstance(node, ast.Name):
            used.add(node.id)
        elif isinstance(node, ast.Attribute):
            base = node
            while isinstance(base, ast.Attribute):
                base = base.value  # type: ignore[assignment]
            if isinstance(base, ast.Name):
                used.add(base.id)
    # names listed in __all__ or used in string annotations count as used
    text = '\n'.join(lines)
    out = []
    for name, lineno in imported.items():
        if name in used or 'noqa' in lines[lineno - 1]:
            continue
        if f"'{name}'" in text or f'"{name}"' in text:
            continue
        out.append((lineno, f'unused import {name!r}'))
    return out


def lint_python(path: str) -> list[str]:
    with open(path, encoding='utf-8') as f:
        src = f.read()
    lines = src.splitlines()
    rel = os.path.relpath(path, ROOT)
    problems = []
    try:
        tree = ast.parse(src, filename=path)
    except SyntaxError as e:
        return [f'{rel}:{e.lineno}: syntax error: {e.msg}']
    if not rel.endswith('__init__.py'):
        problems += [f'{rel}:{n}: {m}' for n, m in _unused_imports(tree, lines)]
    for i, line in enumerate(lines, 1):
        if '\t' in line:
            problems.append(f'{rel}:{i}: tab')
        if line.rstrip() != line:
            problems.append(f'{rel}:{i}: trailing whitespace')
        if len(line) > MAX_LINE and 'http' not in line and 'noqa' not in line:
            problems.append(f'{rel}:{i}: line longer than {MAX_LINE}')
    return problems


def lint_native(path: str) -> list[str]:
    rel = os.path.relpath(path, ROOT)
    problems = []
    with open(path, encoding='utf-8') as f:
        for i, line in enumerate(f.read().splitlines(), 1):
            if '\t' in line:
                problems.append(f'{rel}:{i}: tab')
            if line.rstrip() != line:
                problems.append(f'{rel}:{i}: trailing whitespace')
    return problems


def files() -> tuple[list[str], list[str]]:
    py, native = [os.path.join(ROOT, f) for f in PY_FILES], []
    for d in PY_DIRS + NATIVE_DIRS:
        for dp, _, fs in os.walk(os.path.join(ROOT, d)):
            if '__pycache__' in dp:
                continue
            for f in fs:
                p = os.path.join(dp, f)
                if f.endswith('.py'):
                    py.append(p)
                elif f.endswith(('.hip', '.cpp', '.h')):
                    native.append(p)
    return [p for p in py if os.path.exists(p)], native


def main(argv: list[str]) -> int:
    py, native = files()
    if argv:
        sel = [os.path.abspath(a) for a in argv]
        py = [p for p in py if any(p.startswith(s) for s in sel)]
        native = [p for p in native if any(p.startswith(s) for s in sel)]
    problems = [m for p in py for m in lint_python(p)]
    problems += [m for p in native for m in lint_native(p)]
    for m in problems:
        print(m)
    print(f'{len(py)} python + {len(native)} native files, {len(problems)} findings')
    return 1 if problems else 0


if __name__ == '__main__':
    sys.exit(main(sys.argv[1:]))
