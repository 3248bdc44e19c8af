"""Loss plugins (reference nemo/collections/asr/losses)."""
from nemo.collections.asr.losses.ctc import CTCLoss  # noqa: F401
from nemo.collections.asr.losses.rnnt import RNNTLoss  # noqa: F401
