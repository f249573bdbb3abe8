"""K-FAC beats the first-order baseline (reference integration test)."""
from tests.integration.synthetic_integration import run


def test_kfac_beats_adadelta():
    base, kfac_acc = run(epochs=3, n_train=10_000, n_test=2_000)
    assert kfac_acc > base + 5.0, (base, kfac_acc)
