"""Model shells the reference yamls instantiate (reference nemo/collections/asr/models/__init__.py)."""
from nemo.collections.asr.models.ctc_models import EncDecCTCModel, EncDecCTCModelBPE  # noqa: F401
from nemo.collections.asr.models.rnnt_models import EncDecRNNTBPEModel, EncDecRNNTModel  # noqa: F401
