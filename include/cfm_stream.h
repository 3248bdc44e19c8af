/*
 * cfm_stream.h — C-ABI of the buffered-streaming front end (libcfm.so), SURVEY §8 row a-ext5
 * (BASELINE config 5: Conformer-XLarge, 400-frame buffers advanced by 160-frame chunks, B=64).
 *
 * Replaces, per streaming step, the host numpy work of
 *   FeatureFrameBufferer.get_frame_buffers / _update_feature_buffer / get_norm_consts_per_frame /
 *   normalize_frame_buffers                       (streaming_utils.py:516-549, eps 1e-5)
 *   BatchedFeatureFrameBufferer.get_frame_buffers / _update_feature_buffer / get_norm_consts_per_frame /
 *   normalize_frame_buffers                       (streaming_utils.py:757-806, eps 1e-8)
 * The reference keeps two identical shift-and-append buffers (`buffer`, `feature_buffer`, both
 * total_buffer_len wide and fed the same frames), so one device buffer per stream carries both.
 *
 * For stream s with prev = buffer[s] (F, Tbuf) and new chunks frames[s] (F, k*n):
 *   src = concat(prev, frames[s]) along time;  window_i = src[:, (i+1)*n : (i+1)*n + Tbuf]
 *   out[s*k + i] = (window_i - mean_t(window_i)) / (std_t(window_i) + eps)     (population std)
 *   buffer[s] <- window_{k-1}
 * A stream with active[s] == 0 (the batched reference's `None` frame, streaming_utils.py:775-779,
 * 797-798) has its buffer zeroed and emits an all-zero normalised buffer (k must be 1 then).
 *
 * Conventions as in cfm_encoder.h: device pointers, fp32, status codes + cfm_last_error(),
 * stream-ordered (void* = hipStream_t), no host synchronisation, nothing allocated.
 */
#ifndef CFM_STREAM_H_
#define CFM_STREAM_H_

#include <stddef.h>
#include <stdint.h>

#include "cfm_encoder.h"

#ifdef __cplusplus
extern "C" {
#endif

/* buffer (S, F, Tbuf) in/out; frames (S, F, k*n_frame); active (S) uint8 or NULL (= all active);
 * out (S*k, F, Tbuf) normalised buffers (may be the encoder's audio_signal input).
 * Limits: 1 <= n_frame <= Tbuf, Tbuf + k*n_frame <= 8192. */
cfm_status cfm_frame_buffer_step(float* buffer, const float* frames, const uint8_t* active, int S, int F, int Tbuf,
                                 int n_frame, int k, float eps, float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CFM_STREAM_H_ */
