/*
 * cfm_mel.h — C-ABI of the MI355X-native log-mel front end (libcfm.so), SURVEY §8 row f1: the step
 * before the encoder (conformer_ctc_bpe.yaml:78-92 preprocessor block).
 *
 * Replaces the arithmetic behind
 *   nemo.collections.asr.modules.AudioToMelSpectrogramPreprocessor.forward()  (audio_preprocessing.py:86-90, 276-277)
 *   FilterbankFeatures.forward()                                              (features.py:382-453)
 *       [exact_pad reflect pad] -> [dither, training only] -> pre-emphasis -> torch.stft (center reflect pad,
 *       window zero-padded to n_fft) -> |X| -> |X|^mag_power -> fb @ . -> log(. + guard) | log(clamp(., guard))
 *       -> normalize_batch -> mask t >= seq_len to pad_value -> pad the time axis to a multiple of pad_to
 *   FilterbankFeatures.get_seq_len()                                          (features.py:368-376)
 *   normalize_batch()                                                         (features.py:54-83)
 * The window and mel filterbank are the module's registered buffers (`featurizer.window`,
 * `featurizer.fb`), handed over by cfm_mel_set_tables so checkpoint values are honoured;
 * cfm_mel_filterbank_slaney() restates librosa.filters.mel (Slaney scale + area norm, the
 * reference's features.py:311-314 call) for the initial table.
 *
 * Conventions as in cfm_encoder.h: device pointers, fp32 samples/features, int64 lengths (torch
 * LongTensor), status codes + cfm_last_error(), stream-ordered (void* = hipStream_t), no host sync.
 */
#ifndef CFM_MEL_H_
#define CFM_MEL_H_

#include <stddef.h>
#include <stdint.h>

#include "cfm_encoder.h"

#ifdef __cplusplus
extern "C" {
#endif

#define CFM_NORM_NONE 0
#define CFM_NORM_PER_FEATURE 1
#define CFM_NORM_ALL_FEATURES 2

#define CFM_LOG_GUARD_ADD 0
#define CFM_LOG_GUARD_CLAMP 1

typedef struct cfm_mel cfm_mel;

typedef struct cfm_mel_cfg {
  int n_window_size;     /* win_length (samples) */
  int n_window_stride;   /* hop_length (samples) */
  int n_fft;             /* power of two, 64..4096, >= n_window_size */
  int nfilt;             /* mel bins */
  int exact_pad;         /* 1: reflect-pad (n_fft - hop)/2 before everything, stft center=False */
  int use_preemph;       /* 0: preemph=None */
  float preemph;
  float mag_power;
  int log;               /* 0: no log */
  int log_zero_guard_type;   /* CFM_LOG_GUARD_* */
  float log_zero_guard_value;
  int normalize;         /* CFM_NORM_* */
  float pad_value;
  int pad_to;            /* > 0: multiple; 0: none; -1: "max" (pad to max_length) */
  int max_length;        /* used when pad_to == -1 */
} cfm_mel_cfg;

cfm_status cfm_mel_create(const cfm_mel_cfg* cfg, int device, cfm_mel** out);
void cfm_mel_destroy(cfm_mel* h);
/* window: (n_window_size) fp32, or NULL for 'none' (all ones); fb: (nfilt, n_fft/2+1) fp32.  Device
 * pointers; the library keeps private copies (the filterbank compacted to its nonzero band). */
cfm_status cfm_mel_set_tables(cfm_mel* h, const float* window, const float* fb, void* stream);
/* STFT frames of a padded batch of n_samples, and the output time extent after pad_to. */
long cfm_mel_num_frames(const cfm_mel* h, long n_samples);
long cfm_mel_output_frames(const cfm_mel* h, long n_samples);
/* x (B, N) fp32, len (B) int64 samples -> out (B, nfilt, cfm_mel_output_frames(N)) fp32 and
 * out_len (B) int64 = get_seq_len(len).  dither > 0 adds dither * N(0,1) noise from a counter-based
 * generator keyed by (seed, b, sample) (training only; the caller decides).  nb_mask (B) uint8 or
 * NULL: utterances whose spectrum bins >= nb_max_bin are zeroed (narrow-band augmentation). */
cfm_status cfm_mel_forward(cfm_mel* h, const float* x, const int64_t* len, int B, long N, float dither, uint64_t seed,
                           const uint8_t* nb_mask, int nb_max_bin, float* out, int64_t* out_len, void* stream);
/* normalize_batch(x, seq_len, type) for type per_feature / all_features: (x - mean) / (std + 1e-5)
 * with torch's unbiased std over t < seq_len[b]; x (B, F, T) -> out (may alias x). */
cfm_status cfm_normalize_batch(const float* x, const int64_t* seq_len, int B, int F, int T, int type, float* out,
                               void* stream);
/* Host helper: librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax, htk, norm='slaney' if slaney_norm)
 * into out (n_mels, n_fft/2+1) row-major fp32. */
cfm_status cfm_mel_filterbank_slaney(int sample_rate, int n_fft, int n_mels, double fmin, double fmax, int htk,
                                     int slaney_norm, float* out);

#ifdef __cplusplus
}
#endif
#endif /* CFM_MEL_H_ */
