"""WER metrics (reference nemo/collections/asr/metrics)."""
from nemo.collections.asr.metrics.wer import RNNTWER, WER, word_error_rate  # noqa: F401
