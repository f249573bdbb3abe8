"""Warning categories (reference ``kfac/warnings.py:1-8``)."""
from __future__ import annotations


class ExperimentalFeatureWarning(Warning):
    """Raised when an experimental code path (e.g. the TP/PP preconditioner)
    is used."""
