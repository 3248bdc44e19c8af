"""`EncDecRNNTModel` / `EncDecRNNTBPEModel` (reference nemo/collections/asr/models/rnnt_models.py:59-126,
620-760; rnnt_bpe_models.py) over the MI355X-native drop-ins: mel preprocessor, SpecAugment,
ConformerEncoder, RNNTDecoder (prediction net), RNNTJoint, RNNTLoss and greedy decoding, all in
libcfm.so.

Same construction: decoder.vocab_size and joint.num_classes / vocabulary from `labels` (char) or the
tokenizer (BPE), joint.jointnet.encoder_hidden / pred_hidden from `model_defaults`, RNNTLoss from
the `loss:` block, greedy decoding from `decoding:`, the fused joint step wired when
`joint.fuse_loss_wer` is set (rnnt_models.py:117-122).  `forward` is the encoder step (returns
(encoded, encoded_len)); `training_step` / `validation_step` run prediction net + joint + loss (fused or
not) and the WER; under autograd every stage has a native backward (encoder: cfm_train.h; prediction
net and joint: the training sections of cfm_rnnt_decode.h / cfm_joint.h; loss: cfm_rnnt_loss.h).
Beam / TSD / ALSD decoding strategies are out of scope.
"""
from __future__ import annotations

from typing import List, Optional

import torch

from nemo.collections.asr.losses.rnnt import RNNTLoss
from nemo.collections.asr.metrics.wer import RNNTWER
from nemo.collections.asr.parts.mixins import ASRBPEMixin
from nemo.collections.asr.parts.submodules.rnnt_greedy_decoding import GreedyBatchedRNNTInfer, GreedyRNNTInfer
from nemo.core.classes.common import typecheck
from nemo.core.classes.modelPT import ModelPT
from nemo.core.config import Config
from nemo.core.neural_types import (AcousticEncodedRepresentation, AudioSignal, LengthsType, NeuralType,
                                    SpectrogramType)


class RNNTDecoding:
    """rnnt_wer.py RNNTDecoding for strategy greedy | greedy_batch (the transducer yamls' value)."""

    def __init__(self, decoding_cfg, decoder, joint, vocabulary=None, tokenizer=None):
        cfg = decoding_cfg or {}
        self.strategy = cfg.get("strategy", "greedy_batch")
        blank = joint.num_classes_with_blank - 1
        greedy = cfg.get("greedy", {}) or {}
        max_symbols = greedy.get("max_symbols", None)
        self.joint_fused_batch_size = cfg.get("fused_batch_size", None)
        if self.strategy == "greedy":
            self.decoding = GreedyRNNTInfer(decoder_model=decoder, joint_model=joint, blank_index=blank,
                                            max_symbols_per_step=max_symbols)
        elif self.strategy == "greedy_batch":
            self.decoding = GreedyBatchedRNNTInfer(decoder_model=decoder, joint_model=joint, blank_index=blank,
                                                   max_symbols_per_step=max_symbols)
        else:
            raise NotImplementedError(f"decoding strategy {self.strategy!r} (beam search) is out of scope; "
                                      "use greedy or greedy_batch")
        labels = list(vocabulary or [])
        self.decode_tokens_to_str = (tokenizer.ids_to_text if tokenizer is not None
                                     else (lambda ids: "".join(labels[i] for i in ids)))

    def __call__(self, encoder_output, encoded_lengths):
        return self.decoding(encoder_output=encoder_output, encoded_lengths=encoded_lengths)

    def rnnt_decoder_predictions_tensor(self, encoder_output: torch.Tensor, encoded_lengths: torch.Tensor) -> List[str]:
        with torch.no_grad():
            (hyps,) = self.decoding(encoder_output=encoder_output, encoded_lengths=encoded_lengths)
        return [self.decode_tokens_to_str([int(t) for t in h.y_sequence]) for h in hyps]


class EncDecRNNTModel(ModelPT):
    def __init__(self, cfg, trainer=None):
        super().__init__(cfg=cfg, trainer=trainer)
        cfg = self._cfg
        self.world_size = 1 if trainer is None else getattr(trainer, "world_size", 1)
        self.preprocessor = EncDecRNNTModel.from_config_dict(cfg.preprocessor)
        self.encoder = EncDecRNNTModel.from_config_dict(cfg.encoder)
        labels = list(cfg.labels)
        cfg.decoder["vocab_size"] = len(labels)
        cfg.joint["num_classes"] = len(labels)
        cfg.joint["vocabulary"] = labels
        cfg.joint.jointnet["encoder_hidden"] = cfg.model_defaults.enc_hidden
        cfg.joint.jointnet["pred_hidden"] = cfg.model_defaults.pred_hidden
        self.decoder = EncDecRNNTModel.from_config_dict(cfg.decoder)
        self.joint = EncDecRNNTModel.from_config_dict(cfg.joint)
        loss_cfg = cfg.get("loss", None) or {}
        loss_name = loss_cfg.get("loss_name", "default")
        loss_kwargs = loss_cfg.get(f"{'warprnnt_numba' if loss_name == 'default' else loss_name}_kwargs", None)
        self.loss = RNNTLoss(num_classes=self.joint.num_classes_with_blank - 1, loss_name=loss_name,
                             loss_kwargs=dict(loss_kwargs) if loss_kwargs else None)
        if cfg.get("spec_augment") is not None:
            self.spec_augmentation = EncDecRNNTModel.from_config_dict(cfg.spec_augment)
        else:
            self.spec_augmentation = None
        self.decoding = self._make_decoding()
        self.wer = RNNTWER(decoding=self.decoding, vocabulary=self.joint.vocabulary,
                           tokenizer=getattr(self, "tokenizer", None), batch_dim_index=0,
                           use_cer=cfg.get("use_cer", False), log_prediction=cfg.get("log_prediction", True),
                           dist_sync_on_step=True)
        self.compute_eval_loss = cfg.get("compute_eval_loss", True)
        if self.joint.fuse_loss_wer or (self.decoding.joint_fused_batch_size or 0) > 0:
            self.joint.set_loss(self.loss)
            self.joint.set_wer(self.wer)

    def _make_decoding(self):
        return RNNTDecoding(decoding_cfg=self._cfg.get("decoding", None), decoder=self.decoder, joint=self.joint,
                            vocabulary=self.joint.vocabulary)

    @property
    def input_types(self):
        sr = getattr(self.preprocessor, "_sample_rate", None)
        return {"input_signal": NeuralType(("B", "T"), AudioSignal(freq=sr), optional=True),
                "input_signal_length": NeuralType(tuple("B"), LengthsType(), optional=True),
                "processed_signal": NeuralType(("B", "D", "T"), SpectrogramType(), optional=True),
                "processed_signal_length": NeuralType(tuple("B"), LengthsType(), optional=True)}

    @property
    def output_types(self):
        return {"outputs": NeuralType(("B", "D", "T"), AcousticEncodedRepresentation()),
                "encoded_lengths": NeuralType(tuple("B"), LengthsType())}

    @typecheck()
    def forward(self, input_signal=None, input_signal_length=None, processed_signal=None,
                processed_signal_length=None):
        """rnnt_models.py:620-670: the acoustic-model step only."""
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
        return self.encoder(audio_signal=processed_signal, length=processed_signal_length)

    def _forward_batch(self, batch, processed: bool):
        signal, signal_len = batch[0], batch[1]
        if processed:
            return self.forward(processed_signal=signal, processed_signal_length=signal_len)
        return self.forward(input_signal=signal, input_signal_length=signal_len)

    def _loss_and_wer(self, encoded, encoded_len, transcript, transcript_len, compute_wer: bool):
        decoder, target_length, _ = self.decoder(targets=transcript, target_length=transcript_len)
        if not self.joint.fuse_loss_wer:
            joint = self.joint(encoder_outputs=encoded, decoder_outputs=decoder)
            loss_value = self.loss(log_probs=joint, targets=transcript, input_lengths=encoded_len,
                                   target_lengths=target_length)
            wer = wer_num = wer_denom = None
            if compute_wer:
                self.wer.update(encoded, encoded_len, transcript, transcript_len)
                wer, wer_num, wer_denom = self.wer.compute()
                self.wer.reset()
            return loss_value, wer, wer_num, wer_denom
        return self.joint(encoder_outputs=encoded, decoder_outputs=decoder, encoder_lengths=encoded_len,
                          transcripts=transcript, transcript_lengths=transcript_len, compute_wer=compute_wer)

    def training_step(self, batch, batch_nb, processed_signal: bool = False):
        """rnnt_models.py:673-739: encoder forward, prediction net on the transcripts, then the joint + RNN-T
        loss (fused in sub-batches when fuse_loss_wer, rnnt.py:824-949); loss.backward() runs the native
        RNN-T loss gradient, joint backward, prediction-net BPTT and the encoder's native backward."""
        _, _, transcript, transcript_len = batch[:4]
        encoded, encoded_len = self._forward_batch(batch, processed_signal)
        every = getattr(self._trainer, "log_every_n_steps", 1) if self._trainer is not None else 1
        compute_wer = (batch_nb + 1) % every == 0
        loss_value, wer, _, _ = self._loss_and_wer(encoded, encoded_len, transcript, transcript_len, compute_wer)
        logs = {"train_loss": loss_value, "learning_rate": self._current_lr()}
        if compute_wer:
            logs["training_batch_wer"] = wer
        return {"loss": loss_value, "log": logs}

    @torch.no_grad()
    def validation_step(self, batch, batch_idx, dataloader_idx=0, processed_signal: bool = False):
        """rnnt_models.py:760-800."""
        _, _, transcript, transcript_len = batch[:4]
        encoded, encoded_len = self._forward_batch(batch, processed_signal)
        out = {}
        if self.compute_eval_loss:
            loss_value, wer, wer_num, wer_denom = self._loss_and_wer(encoded, encoded_len, transcript,
                                                                     transcript_len, True)
            out["val_loss"] = loss_value
        else:
            self.wer.update(encoded, encoded_len, transcript, transcript_len)
            wer, wer_num, wer_denom = self.wer.compute()
            self.wer.reset()
        out.update({"val_wer_num": wer_num, "val_wer_denom": wer_denom, "val_wer": wer})
        return out

    @torch.no_grad()
    def transcribe_processed(self, processed_signal: torch.Tensor, processed_signal_length: torch.Tensor) -> List[str]:
        """`transcribe` minus audio-file loading: greedy hypotheses of a batch of spectrograms."""
        mode = self.training
        self.eval()
        try:
            encoded, encoded_len = self.forward(processed_signal=processed_signal,
                                                processed_signal_length=processed_signal_length)
            return self.decoding.rnnt_decoder_predictions_tensor(encoded, encoded_len)
        finally:
            self.train(mode)


class EncDecRNNTBPEModel(EncDecRNNTModel, ASRBPEMixin):
    """rnnt_bpe_models.py: the tokenizer's vocabulary becomes `labels`."""

    def __init__(self, cfg, trainer=None):
        if not isinstance(cfg, Config):
            cfg = Config(cfg)
        if "model" in cfg and "encoder" not in cfg:
            cfg = cfg.model
        if "tokenizer" not in cfg:
            raise ValueError("`cfg` must have `tokenizer` config to create a tokenizer !")
        self._setup_tokenizer(cfg.tokenizer)
        cfg["labels"] = self._tokenizer_vocabulary()
        super().__init__(cfg=cfg, trainer=trainer)

    def __setattr__(self, name, value):
        if name in ("tokenizer", "tokenizer_dir", "tokenizer_type") and "_modules" not in self.__dict__:
            object.__setattr__(self, name, value)
        else:
            super().__setattr__(name, value)

    def _make_decoding(self):
        return RNNTDecoding(decoding_cfg=self._cfg.get("decoding", None), decoder=self.decoder, joint=self.joint,
                            tokenizer=self.tokenizer)
