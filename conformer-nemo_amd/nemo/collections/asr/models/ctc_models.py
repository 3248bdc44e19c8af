"""`EncDecCTCModel` / `EncDecCTCModelBPE` (reference nemo/collections/asr/models/ctc_models.py:161-630,
ctc_bpe_models.py:220-263): the model shells `conformer_ctc_char.yaml` / `conformer_ctc_bpe.yaml`
instantiate, over the MI355X-native drop-ins (mel preprocessor, SpecAugment, ConformerEncoder,
ConvASRDecoder, CTCLoss — every one running in libcfm.so).

Same construction (sub-modules by `from_config_dict` from the config blocks, decoder.feat_in from
the encoder's `_feat_out`, num_classes from the vocabulary, CTCLoss(num_classes, zero_infinity=True,
reduction=ctc_reduction)), same keyword-only `forward` (raw audio through the preprocessor, or
`processed_signal`; SpecAugment only in training; returns (log_probs, encoded_len,
greedy_predictions)), same `training_step` / `validation_step` dictionaries.  Lightning's trainer,
data loaders and `transcribe` from audio files are out of scope; a training loop calls
`training_step(batch, i)['loss'].backward()` and the optimizer `setup_optimization` built.
"""
from __future__ import annotations

from typing import Optional

import torch

from nemo.collections.asr.losses.ctc import CTCLoss
from nemo.collections.asr.metrics.wer import WER
from nemo.collections.asr.parts.mixins import ASRBPEMixin
from nemo.core.classes.common import typecheck
from nemo.core.classes.modelPT import ModelPT
from nemo.core.config import Config
from nemo.core.neural_types import (AcousticEncodedRepresentation, AudioSignal, LabelsType, LengthsType,
                                    LogprobsType, NeuralType, SpectrogramType)


class EncDecCTCModel(ModelPT):
    """ctc_models.py:161-212 (construction), 527-596 (types, forward), 599-680 (steps)."""

    def __init__(self, cfg, trainer=None):
        super().__init__(cfg=cfg, trainer=trainer)
        cfg = self._cfg
        self.world_size = 1 if trainer is None else getattr(trainer, "world_size", 1)
        self.preprocessor = EncDecCTCModel.from_config_dict(cfg.preprocessor)
        self.encoder = EncDecCTCModel.from_config_dict(cfg.encoder)
        dec = cfg.decoder
        if "feat_in" not in dec or (not dec.get("feat_in") and hasattr(self.encoder, "_feat_out")):
            dec["feat_in"] = self.encoder._feat_out
        if not dec.get("feat_in"):
            raise ValueError("param feat_in of the decoder's config is not set!")
        if dec.get("num_classes", -1) < 1 and dec.get("vocabulary") is not None:
            dec["num_classes"] = len(dec["vocabulary"])
        self.decoder = EncDecCTCModel.from_config_dict(dec)
        self.loss = CTCLoss(num_classes=self.decoder.num_classes_with_blank - 1, zero_infinity=True,
                            reduction=cfg.get("ctc_reduction", "mean_batch"))
        if cfg.get("spec_augment") is not None:
            self.spec_augmentation = EncDecCTCModel.from_config_dict(cfg.spec_augment)
        else:
            self.spec_augmentation = None
        self._wer = self._make_wer()

    def _make_wer(self):
        return WER(vocabulary=self.decoder.vocabulary, batch_dim_index=0, use_cer=self._cfg.get("use_cer", False),
                   ctc_decode=True, dist_sync_on_step=True, log_prediction=self._cfg.get("log_prediction", False))

    @property
    def wer(self):
        return self._wer

    @property
    def input_types(self):
        sr = getattr(self.preprocessor, "_sample_rate", None)
        return {"input_signal": NeuralType(("B", "T"), AudioSignal(freq=sr), optional=True),
                "input_signal_length": NeuralType(tuple("B"), LengthsType(), optional=True),
                "processed_signal": NeuralType(("B", "D", "T"), SpectrogramType(), optional=True),
                "processed_signal_length": NeuralType(tuple("B"), LengthsType(), optional=True),
                "sample_id": NeuralType(tuple("B"), LengthsType(), optional=True)}

    @property
    def output_types(self):
        return {"outputs": NeuralType(("B", "T", "D"), LogprobsType()),
                "encoded_lengths": NeuralType(tuple("B"), LengthsType()),
                "greedy_predictions": NeuralType(("B", "T"), LabelsType())}

    @typecheck()
    def forward(self, input_signal=None, input_signal_length=None, processed_signal=None,
                processed_signal_length=None):
        has_input = input_signal is not None and input_signal_length is not None
        has_processed = processed_signal is not None and processed_signal_length is not None
        if (has_input ^ has_processed) is False:
            raise ValueError(f"{self} Arguments ``input_signal`` and ``input_signal_length`` are mutually exclusive "
                             " with ``processed_signal`` and ``processed_signal_len`` arguments.")
        if not has_processed:
            processed_signal, processed_signal_length = self.preprocessor(input_signal=input_signal,
                                                                          length=input_signal_length)
        if self.spec_augmentation is not None and self.training:
            processed_signal = self.spec_augmentation(input_spec=processed_signal, length=processed_signal_length)
        encoded, encoded_len = self.encoder(audio_signal=processed_signal, length=processed_signal_length)
        log_probs = self.decoder(encoder_output=encoded)
        greedy_predictions = log_probs.argmax(dim=-1, keepdim=False)
        return log_probs, encoded_len, greedy_predictions

    def _forward_batch(self, batch, processed: bool):
        signal, signal_len = batch[0], batch[1]
        if processed:
            return self.forward(processed_signal=signal, processed_signal_length=signal_len)
        return self.forward(input_signal=signal, input_signal_length=signal_len)

    def training_step(self, batch, batch_nb, processed_signal: bool = False):
        """ctc_models.py:599-630.  batch = (signal, signal_len, transcript, transcript_len); with
        processed_signal=True the signal is a (B, D, T) spectrogram (the reference's DALI branch)."""
        _, _, transcript, transcript_len = batch[:4]
        log_probs, encoded_len, predictions = self._forward_batch(batch, processed_signal)
        loss_value = self.loss(log_probs=log_probs, targets=transcript, input_lengths=encoded_len,
                               target_lengths=transcript_len)
        logs = {"train_loss": loss_value, "learning_rate": self._current_lr()}
        every = getattr(self._trainer, "log_every_n_steps", 1) if self._trainer is not None else 1
        if (batch_nb + 1) % every == 0:
            self._wer.update(predictions=predictions, targets=transcript, target_lengths=transcript_len,
                             predictions_lengths=encoded_len)
            wer, _, _ = self._wer.compute()
            self._wer.reset()
            logs["training_batch_wer"] = wer
        return {"loss": loss_value, "log": logs}

    def validation_step(self, batch, batch_idx, dataloader_idx=0, processed_signal: bool = False):
        """ctc_models.py:650-667."""
        _, _, transcript, transcript_len = batch[:4]
        log_probs, encoded_len, predictions = self._forward_batch(batch, processed_signal)
        loss_value = self.loss(log_probs=log_probs, targets=transcript, input_lengths=encoded_len,
                               target_lengths=transcript_len)
        self._wer.update(predictions=predictions, targets=transcript, target_lengths=transcript_len,
                         predictions_lengths=encoded_len)
        wer, wer_num, wer_denom = self._wer.compute()
        self._wer.reset()
        return {"val_loss": loss_value, "val_wer_num": wer_num, "val_wer_denom": wer_denom, "val_wer": wer}

    def test_step(self, batch, batch_idx, dataloader_idx=0, processed_signal: bool = False):
        logs = self.validation_step(batch, batch_idx, dataloader_idx, processed_signal)
        return {name.replace("val_", "test_"): value for name, value in logs.items()}

    @torch.no_grad()
    def transcribe_processed(self, processed_signal: torch.Tensor, processed_signal_length: torch.Tensor):
        """`transcribe` (ctc_models.py:214-300) minus audio-file loading: greedy CTC hypotheses of a
        batch of spectrograms."""
        mode = self.training
        self.eval()
        try:
            _, encoded_len, predictions = self.forward(processed_signal=processed_signal,
                                                       processed_signal_length=processed_signal_length)
            return self._wer.ctc_decoder_predictions_tensor(predictions, predictions_len=encoded_len)
        finally:
            self.train(mode)


class EncDecCTCModelBPE(EncDecCTCModel, ASRBPEMixin):
    """ctc_bpe_models.py:220-263: the tokenizer's vocabulary becomes decoder.vocabulary (and
    num_classes when the config leaves the -1 placeholder)."""

    def __init__(self, cfg, trainer=None):
        if not isinstance(cfg, Config):
            cfg = Config(cfg)
        if "model" in cfg and "encoder" not in cfg:
            cfg = cfg.model
        if "tokenizer" not in cfg:
            raise ValueError("`cfg` must have `tokenizer` config to create a tokenizer !")
        self._setup_tokenizer(cfg.tokenizer)
        vocabulary = self._tokenizer_vocabulary()
        cfg.decoder["vocabulary"] = vocabulary
        if cfg.decoder.get("num_classes", -1) < 1:
            cfg.decoder["num_classes"] = len(vocabulary)
        super().__init__(cfg=cfg, trainer=trainer)

    def __setattr__(self, name, value):
        # the tokenizer is set before nn.Module.__init__ runs (as in the reference)
        if name in ("tokenizer", "tokenizer_dir", "tokenizer_type") and "_modules" not in self.__dict__:
            object.__setattr__(self, name, value)
        else:
            super().__setattr__(name, value)

    def _make_wer(self):
        return WER(tokenizer=self.tokenizer, batch_dim_index=0, use_cer=self._cfg.get("use_cer", False),
                   ctc_decode=True, dist_sync_on_step=True, log_prediction=self._cfg.get("log_prediction", False))
