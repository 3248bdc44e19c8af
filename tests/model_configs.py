"""Small model configs written in the reference yamls' dialect (anchors, `${}` interpolation, `???`
markers, the same block names and keys as configs/conformer_{ctc,transducer}_bpe.yaml) at test
sizes, for the model-shell tests on boxes without /root/reference; and a helper that trains a tiny
SentencePiece BPE tokenizer (the `tokenizer.dir` those configs require)."""
import os

REF_CONFIGS = "/root/reference/configs"

CTC_BPE_SMALL = """
name: "Conformer-CTC-BPE-test"
model:
  sample_rate: &sample_rate 16000
  log_prediction: true
  ctc_reduction: 'mean_batch'
  train_ds:
    manifest_filepath: ???
    sample_rate: ${model.sample_rate}
    batch_size: 4
  tokenizer:
    dir: ???
    type: bpe
  preprocessor:
    _target_: nemo.collections.asr.modules.AudioToMelSpectrogramPreprocessor
    sample_rate: *sample_rate
    normalize: "per_feature"
    window_size: 0.025
    window_stride: 0.01
    window: "hann"
    features: 80
    n_fft: 512
    log: true
    frame_splicing: 1
    dither: 0.0
    pad_to: 0
    pad_value: 0.0
  spec_augment:
    _target_: nemo.collections.asr.modules.SpectrogramAugmentation
    freq_masks: 2
    time_masks: 2
    freq_width: 27
    time_width: 0.05
  encoder:
    _target_: nemo.collections.asr.modules.ConformerEncoder
    feat_in: ${model.preprocessor.features}
    feat_out: -1
    n_layers: 2
    d_model: 128
    subsampling: striding
    subsampling_factor: 4
    subsampling_conv_channels: -1
    ff_expansion_factor: 4
    self_attention_model: rel_pos
    n_heads: 4
    att_context_size: [-1, -1]
    xscaling: true
    untie_biases: true
    pos_emb_max_len: 5000
    conv_kernel_size: 31
    conv_norm_type: 'batch_norm'
    dropout: 0.1
    dropout_emb: 0.0
    dropout_att: 0.1
  decoder:
    _target_: nemo.collections.asr.modules.ConvASRDecoder
    feat_in: null
    num_classes: -1
    vocabulary: []
  optim:
    name: adamw
    lr: 2.0
    betas: [0.9, 0.98]
    weight_decay: 1e-3
    sched:
      name: NoamAnnealing
      d_model: ${model.encoder.d_model}
      warmup_steps: 10
      warmup_ratio: null
      min_lr: 1e-6
trainer:
  devices: -1
  sync_batchnorm: true
exp_manager:
  name: ${name}
"""

RNNT_BPE_SMALL = """
name: "Conformer-Transducer-BPE-test"
model:
  sample_rate: &sample_rate 16000
  compute_eval_loss: true
  log_prediction: true
  model_defaults:
    enc_hidden: ${model.encoder.d_model}
    pred_hidden: 64
    joint_hidden: 64
  train_ds:
    manifest_filepath: ???
    sample_rate: ${model.sample_rate}
  tokenizer:
    dir: ???
    type: bpe
  preprocessor:
    _target_: nemo.collections.asr.modules.AudioToMelSpectrogramPreprocessor
    sample_rate: *sample_rate
    normalize: "per_feature"
    window_size: 0.025
    window_stride: 0.01
    window: "hann"
    features: 80
    n_fft: 512
    frame_splicing: 1
    dither: 0.0
    pad_to: 0
  spec_augment:
    _target_: nemo.collections.asr.modules.SpectrogramAugmentation
    freq_masks: 2
    time_masks: 2
    freq_width: 8
    time_width: 0.01
    specshot_ratio: 0.2
  encoder:
    _target_: nemo.collections.asr.modules.ConformerEncoder
    feat_in: ${model.preprocessor.features}
    feat_out: -1
    n_layers: 2
    d_model: 128
    subsampling: striding
    subsampling_factor: 4
    subsampling_conv_channels: -1
    ff_expansion_factor: 4
    self_attention_model: rel_pos
    n_heads: 4
    att_context_size: [-1, -1]
    xscaling: true
    untie_biases: true
    pos_emb_max_len: 5000
    conv_kernel_size: 31
    conv_norm_type: 'batch_norm'
    dropout: 0.1
    dropout_emb: 0.0
    dropout_att: 0.1
  decoder:
    _target_: nemo.collections.asr.modules.RNNTDecoder
    normalization_mode: null
    random_state_sampling: false
    blank_as_pad: true
    prednet:
      pred_hidden: ${model.model_defaults.pred_hidden}
      pred_rnn_layers: 1
      t_max: null
      dropout: 0.1
  joint:
    _target_: nemo.collections.asr.modules.RNNTJoint
    log_softmax: null
    preserve_memory: false
    fuse_loss_wer: true
    fused_batch_size: 2
    jointnet:
      joint_hidden: ${model.model_defaults.joint_hidden}
      activation: "relu"
      dropout: 0.1
  decoding:
    strategy: "greedy_batch"
    greedy:
      max_symbols: 5
  loss:
    loss_name: "default"
    warprnnt_numba_kwargs:
      fastemit_lambda: 0.0
      clamp: -1.0
  optim:
    name: adamw
    lr: 5.0
    betas: [0.9, 0.98]
    weight_decay: 1e-3
trainer:
  sync_batchnorm: true
"""

_CORPUS = ["the quick brown fox jumps over the lazy dog", "speech recognition with conformer models",
           "hello world this is a test of the transducer", "native kernels on the accelerator"]


def make_bpe_tokenizer(directory: str, vocab_size: int = 40) -> str:
    """Train a tiny SentencePiece BPE model into `directory`/tokenizer.model; returns directory."""
    import sentencepiece as spm
    os.makedirs(directory, exist_ok=True)
    corpus = os.path.join(directory, "corpus.txt")
    with open(corpus, "w", encoding="utf-8") as f:
        f.write("\n".join(_CORPUS * 40))
    spm.SentencePieceTrainer.train(input=corpus, model_prefix=os.path.join(directory, "tokenizer"),
                                   vocab_size=vocab_size, model_type="bpe", character_coverage=1.0,
                                   minloglevel=2)
    return directory
