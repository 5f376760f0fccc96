"""NL->SQL evaluation harness (reproduction of Model_Evaluation_&_Comparision.py).

The functions are re-exported lazily so ``python -m ...eval.harness`` does not import the module twice.
"""

__all__ = ["evaluate_single", "evaluate_multi", "summarize"]


def __getattr__(name):
    if name in __all__:
        from . import harness

        return getattr(harness, name)
    raise AttributeError(name)
