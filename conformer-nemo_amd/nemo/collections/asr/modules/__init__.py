"""Module plugins resolvable by yaml `_target_` (reference nemo/collections/asr/modules)."""
from nemo.collections.asr.modules.conformer_encoder import ConformerEncoder  # noqa: F401
from nemo.collections.asr.modules.conv_asr import ConvASRDecoder  # noqa: F401
from nemo.collections.asr.modules.rnnt import RNNTDecoder, RNNTJoint  # noqa: F401
from nemo.collections.asr.modules.audio_preprocessing import (  # noqa: F401
    AudioToMelSpectrogramPreprocessor, SpectrogramAugmentation)
