"""NL->SQL evaluation harness (reproduction of Model_Evaluation_&_Comparision.py)."""
from .harness import evaluate_single, evaluate_multi, summarize  # noqa: F401
