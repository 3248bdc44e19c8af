/*
 * cfm_cache_stream.h — cache-aware chunked streaming of the Conformer encoder (libcfm.so),
 * SURVEY §8 row f3.
 *
 * The reference streams by re-encoding overlapping 400-frame buffers with the stateless encoder
 * (FeatureFrameBufferer / FrameBatchASR, streaming_utils.py:455-683; built as cfm_stream.h).  60 %
 * of each buffer is recomputed every step.  This entry point instead encodes only the new frames
 * of each chunk and carries the state between chunks on the device:
 *   - the last 2 input (mel) frames and the last 2 conv1 output frames of the subsampling,
 *   - per layer, the keys and values of the last `left_context` encoder frames (after linear_k /
 *     linear_v, so they are not recomputed),
 *   - per layer, the last kernel_size-1 GLU outputs feeding the depthwise convolution.
 *
 * WHAT IT COMPUTES (the definition; the reference has no such model, so parity is unpinned and
 * defined against a full-sequence forward of the same causal encoder, oracle/cache_aware_oracle.py):
 * the reference ConformerEncoder with three changes that make frame t depend on frames <= t only -
 *   (1) both subsampling convolutions pad time by (2, 0) instead of (1, 1) (frequency keeps (1, 1)),
 *   (2) attention context [left_context, 0]: frame i attends to frames max(0, i - left_context) .. i,
 *   (3) the depthwise convolution pads time by (kernel_size - 1, 0) instead of symmetrically.
 * Everything else (weights, state_dict, rel-pos MHSA with pos_bias_u/v, xscale, BatchNorm with
 * running statistics, LayerNorms, macaron FFNs, out_proj) is the reference's.  Under this
 * definition the chunked outputs equal the full-sequence outputs for any chunk size (the test
 * gate: fp32 compute relL2 <= 1e-3 against the numpy oracle; bf16 reported).
 *
 * Conventions as in cfm_encoder.h: device pointers, fp32 in/out, status codes + cfm_last_error(),
 * stream-ordered (void* = hipStream_t), no host synchronisation in cfm_cache_stream_step.
 * The encoder handle supplies the packed weights; it must outlive the stream state, and
 * cfm_cache_stream_reset must be called after cfm_encoder_set_weights.
 */
#ifndef CFM_CACHE_STREAM_H_
#define CFM_CACHE_STREAM_H_

#include <stddef.h>
#include <stdint.h>

#include "cfm_encoder.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cfm_cache_stream cfm_cache_stream;

/* State for `batch` streams advancing `chunk` encoder frames (= 4 * chunk input frames) per step,
 * attending `left_context` encoder frames back.  Requires the striding/4 subsampling (as the
 * encoder), chunk >= 1, 1 <= left_context < pos_emb_max_len.  Allocates the state (device) and
 * builds the per-layer position projections; synchronises nothing. */
cfm_status cfm_cache_stream_create(cfm_encoder* enc, int batch, int chunk, int left_context, cfm_cache_stream** out);
cfm_status cfm_cache_stream_destroy(cfm_cache_stream* s);

/* Zero every cache, restart at frame 0 and rebuild the position projections from the encoder's
 * current weights (stream-ordered). */
cfm_status cfm_cache_stream_reset(cfm_cache_stream* s, void* stream);

/* Bytes of scratch one step needs (caller-owned, like cfm_encoder_workspace_size). */
size_t cfm_cache_stream_workspace_size(const cfm_cache_stream* s);

/* One chunk for every stream: x (batch, feat_in, 4 * chunk) fp32 log-mel frames -> y (batch,
 * d_model or feat_out, chunk) fp32 encoder frames.  Advances the state by `chunk` frames. */
cfm_status cfm_cache_stream_step(cfm_cache_stream* s, const float* x_bft, float* y_bdt, void* workspace,
                                 size_t workspace_bytes, void* stream);

/* Encoder frames emitted so far (host counter). */
int64_t cfm_cache_stream_position(const cfm_cache_stream* s);

#ifdef __cplusplus
}
#endif
#endif
