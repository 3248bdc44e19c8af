/*
 * cfm_rnnt_decode.h — C-ABI of the RNN-T prediction network and greedy batch decoding (libcfm.so),
 * SURVEY §8 rows a-ext4 (RNNTDecoder.predict, the decoder side of config 4) and f2 (greedy batch
 * decoding after the joint).
 *
 * Replaces the arithmetic behind
 *   RNNTDecoder.forward / predict             nemo/collections/asr/modules/rnnt.py:158-283
 *     embedding (blank = padding row) -> [zero SOS step] -> torch.nn.LSTM (LSTMDropout,
 *     nemo/collections/common/parts/rnn.py:151-237; gate order i, f, g, o; eval: no dropout)
 *   GreedyBatchedRNNTInfer._greedy_decode_blank_as_pad
 *                                             nemo/collections/asr/parts/submodules/rnnt_greedy_decoding.py:453-616
 *     with RNNTJoint.joint (rnnt.py:951-1008) at every (frame, symbol) step.
 *
 * Greedy decoding runs per utterance on the device: each utterance keeps its own frame pointer,
 * symbol count, last label and LSTM state, so one "iteration" advances every active utterance by one
 * prediction-net + joint step.  This is exactly the reference's lock-step batch loop, whose masked
 * utterances keep their state and label (rnnt_greedy_decoding.py:557-575): tokens never depend on
 * batch neighbours.  Scores are sums of the selected raw logits (the reference's GPU behaviour,
 * :181-185) or of log-probabilities when log_normalize != 0 (its CPU behaviour).
 *
 * All arithmetic is fp32 (the argmax is discrete: a lower-precision path could flip near-ties).
 * Conventions as in cfm_encoder.h: device pointers, status codes + cfm_last_error(), void* =
 * hipStream_t, caller-owned workspace.  cfm_rnnt_decoder_predict is stream-ordered with no host
 * synchronisation; cfm_rnnt_greedy_decode SYNCHRONISES `stream` (it polls a device done-flag every
 * few iterations to know when every utterance has finished) and returns when decoding is complete.
 */
#ifndef CFM_RNNT_DECODE_H_
#define CFM_RNNT_DECODE_H_

#include <stddef.h>
#include <stdint.h>

#include "cfm_encoder.h"
#include "cfm_joint.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct cfm_rnnt_decoder cfm_rnnt_decoder;

/* vocab_size excludes blank (blank index = vocab_size, the embedding's padding row);
 * pred_hidden = embedding and LSTM width (a multiple of 4, <= 1536); layers = pred_rnn_layers. */
cfm_status cfm_rnnt_decoder_create(int vocab_size, int pred_hidden, int layers, int device, cfm_rnnt_decoder** out);
void cfm_rnnt_decoder_destroy(cfm_rnnt_decoder* h);
/* Reference parameters (device fp32, borrowed): prediction.embed.weight (V+1, H) and per layer l
 * prediction.dec_rnn.lstm.{weight_ih_l, weight_hh_l} (4H, H), {bias_ih_l, bias_hh_l} (4H).
 * Packs private copies ([W_ih | W_hh] rows, b_ih + b_hh) on `stream` (stream-ordered, no host
 * synchronisation: the sources must stay valid until `stream` reaches the call). */
cfm_status cfm_rnnt_decoder_set_weights(cfm_rnnt_decoder* h, const float* embed, const float* const* w_ih,
                                        const float* const* w_hh, const float* const* b_ih,
                                        const float* const* b_hh, void* stream);

/* RNNTDecoder.predict(y, state, add_sos): y (B, U) int64 labels (or NULL: one zero step, the
 * reference's y=None case), h0/c0 (L, B, H) or NULL (zero state) -> g (B, S, H) with
 * S = U' + add_sos (U' = U, or 1 when y is NULL), final h_out/c_out (L, B, H). */
size_t cfm_rnnt_decoder_predict_workspace_size(const cfm_rnnt_decoder* h, int B, int U);
cfm_status cfm_rnnt_decoder_predict(cfm_rnnt_decoder* h, const int64_t* y, int B, int U, int add_sos,
                                    const float* h0, const float* c0, float* g, float* h_out, float* c_out,
                                    void* workspace, size_t workspace_bytes, void* stream);

/* Greedy batch decoding.  enc_bdt (B, D1, T) encoder output, enc_len (B) int64 frame counts
 * (clamped to [0, T]).  Joint parameters (device fp32, borrowed, reference layouts): w_enc (J, D1),
 * b_enc (J), w_pred (J, H), b_pred (J), w_out (V+1, J), b_out (V+1), J % 4 == 0, J <= 3072;
 * activation CFM_JOINT_*.
 * max_symbols >= 1 labels per frame.  sos_until_label = 0: GreedyBatchedRNNTInfer's inputs (zero SOS
 * vector on an utterance's first step, then the embedding of its last label — the blank row while
 * none was emitted); 1: GreedyRNNTInfer's (zero SOS vector until the first label, :315-318).
 * Outputs: tokens / timesteps (B, T*max_symbols) int32 (first
 * ntok[b] entries valid), ntok (B) int32, scores (B) fp64, h_out / c_out (L, B, H) final states. */
size_t cfm_rnnt_greedy_workspace_size(const cfm_rnnt_decoder* h, int B, int T, int J);
cfm_status cfm_rnnt_greedy_decode(cfm_rnnt_decoder* h, const float* enc_bdt, const int64_t* enc_len, int B, int T,
                                  int D1, int J, const float* w_enc, const float* b_enc, const float* w_pred,
                                  const float* b_pred, const float* w_out, const float* b_out, int activation,
                                  int max_symbols, int log_normalize, int sos_until_label, int32_t* tokens,
                                  int32_t* timesteps, int32_t* ntok, double* scores, float* h_out, float* c_out,
                                  void* workspace, size_t workspace_bytes, void* stream);

/* ---- training (RNNTDecoder.predict under autograd, rnnt.py:190-283; rnnt_models.py:673-739) ------ */
/* Teacher-forced prediction network from the zero state: y (B, U) int64 labels (+ the zero SOS step when
 * add_sos) -> g (B, S, H), S = U + add_sos, with LSTMDropout's output Dropout(p = dropout) (rnn.py:151-237;
 * counter-hash mask keyed by seed, regenerated by the backward).  Records a tape (gates, cells, hidden
 * states of every layer and step) of cfm_rnnt_decoder_train_tape_size bytes for the backward. */
size_t cfm_rnnt_decoder_train_tape_size(const cfm_rnnt_decoder* h, int B, int U, int add_sos);
cfm_status cfm_rnnt_decoder_train_forward(cfm_rnnt_decoder* h, const int64_t* y, int B, int U, int add_sos,
                                          float dropout, uint64_t seed, float* g, void* tape, size_t tape_bytes,
                                          void* stream);
/* Backpropagation through time given dg (B, S, H): d_embed (V+1, H) (the blank / padding row and the SOS
 * step get no gradient), per layer dw_ih / dw_hh (4H, H) and db_ih = db_hh (4H); any output pointer (or
 * array) may be NULL, db_hh needs db_ih.  w_ih / w_hh: the reference weights of each layer (fp32).
 * Workspace of cfm_rnnt_decoder_backward_workspace_size bytes.  Deterministic: the embedding gradient
 * row of label v sums the steps labelled v in step order, the recurrent product its 16 row splits in
 * split order (no atomics; bitwise reproducible). */
size_t cfm_rnnt_decoder_backward_workspace_size(const cfm_rnnt_decoder* h, int B, int U, int add_sos);
cfm_status cfm_rnnt_decoder_backward(cfm_rnnt_decoder* h, const int64_t* y, int B, int U, int add_sos, float dropout,
                                     uint64_t seed, const void* tape, const float* dg, const float* const* w_ih,
                                     const float* const* w_hh, float* d_embed, float* const* dw_ih,
                                     float* const* dw_hh, float* const* db_ih, float* const* db_hh, void* workspace,
                                     size_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* CFM_RNNT_DECODE_H_ */
