"""utils.env.getenv: the hot-path knob reader follows run-time changes."""
import os

from distributed_kfac_pytorch_amd.utils.env import getenv


def test_getenv_matches_os_environ(monkeypatch):
    monkeypatch.delenv('KFAC_TEST_KNOB', raising=False)
    assert getenv('KFAC_TEST_KNOB') is None
    assert getenv('KFAC_TEST_KNOB', 'd') == 'd'
    monkeypatch.setenv('KFAC_TEST_KNOB', '1')
    assert getenv('KFAC_TEST_KNOB', 'd') == '1'
    os.environ['KFAC_TEST_KNOB'] = 'café'
    assert getenv('KFAC_TEST_KNOB') == os.environ.get('KFAC_TEST_KNOB')
    monkeypatch.delenv('KFAC_TEST_KNOB')
    assert getenv('KFAC_TEST_KNOB', 'x') == 'x'
    for k, v in list(os.environ.items())[:20]:
        assert getenv(k) == v
