"""Every environment knob the library reads is documented.

The knobs are A/B switches kept next to their measured defaults; the table
in ``tools/README.md`` is their single reference.  A knob read anywhere in
the package, the native sources or the bench without a row there fails this
test."""
from __future__ import annotations

import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_READ = re.compile(r"(?:getenv|environ\.get|environ\[|setdefault)\(?\s*[\"'](KFAC_[A-Z0-9_]+)")


def _sources():
    for top in ('distributed_kfac_pytorch_amd', 'csrc'):
        for dirpath, _, files in os.walk(os.path.join(ROOT, top)):
            for f in files:
                if f.endswith(('.py', '.hip', '.cpp', '.h')):
                    yield os.path.join(dirpath, f)
    yield os.path.join(ROOT, 'bench.py')


def test_every_env_knob_is_documented() -> None:
    used: dict[str, str] = {}
    for path in _sources():
        with open(path, encoding='utf-8') as fh:
            for name in _READ.findall(fh.read()):
                used.setdefault(name, os.path.relpath(path, ROOT))
    with open(os.path.join(ROOT, 'tools', 'README.md'), encoding='utf-8') as fh:
        rows = [ln for ln in fh if ln.startswith('| `KFAC_')]
    documented = {n for ln in rows for n in re.findall(r'`(KFAC_[A-Z0-9_]+)`', ln.split('|')[1])}
    missing = {k: v for k, v in used.items() if k not in documented}
    assert not missing, f'undocumented knobs (add a row to tools/README.md): {missing}'
    assert len(used) >= 30, used  # the scan itself works
