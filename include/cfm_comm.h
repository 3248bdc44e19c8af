/* Data-parallel communication through the C-ABI (cfm_comm_init / cfm_allreduce_grads;
 * §8e: one process per GPU, the gradient all-reduce over RCCL/xGMI, overlapped with the backward).
 *
 * Replaces, for a host that is not Python, what the reference gets from PyTorch Lightning's DDP
 * (trainer strategy: ddp, conformer_ctc_bpe.yaml:160) and torch.nn.SyncBatchNorm
 * (sync_batchnorm: true, :175): a communicator over RCCL, a sum all-reduce usable directly as the
 * SyncBatchNorm callback of cfm_train.h, and gradient buckets whose grad_ready callback all-reduces
 * each Conformer layer's gradients while cfm_train_backward is still enqueueing the earlier layers.
 *
 * RCCL is resolved at cfm_comm_init time (the RCCL already loaded in the process - e.g. PyTorch's -
 * or librccl.so.1), so libcfm.so carries no link-time RCCL dependency.  Every call is stream-ordered
 * and host-sync free; every rank must make the same calls in the same order.
 */
#ifndef CFM_COMM_H
#define CFM_COMM_H

#include <stddef.h>
#include <stdint.h>

#include "cfm_encoder.h"

#ifdef __cplusplus
extern "C" {
#endif

#define CFM_COMM_ID_BYTES 128

typedef struct cfm_comm cfm_comm;
typedef struct cfm_grad_buckets cfm_grad_buckets;

/* Rank 0 creates the id and ships it to the other ranks (any side channel). */
cfm_status cfm_comm_get_unique_id(char unique_id[CFM_COMM_ID_BYTES]);
/* One communicator per process (rank in [0, world)) on `device`. */
cfm_status cfm_comm_init(int rank, int world, const char unique_id[CFM_COMM_ID_BYTES], int device, cfm_comm** out);
cfm_status cfm_comm_destroy(cfm_comm* comm);
int cfm_comm_world(const cfm_comm* comm);

/* In-place SUM of n floats at buf (device) over all ranks, then *= scale (1/world: DDP averaging;
 * 1: plain sum), stream-ordered on `stream`. */
cfm_status cfm_allreduce_grads(cfm_comm* comm, float* buf, int64_t n, float scale, void* stream);
/* cfm_allreduce_fn-compatible trampoline (user = cfm_comm*): SyncBatchNorm statistics in cfm_train.h. */
int cfm_comm_allreduce_cb(void* user, float* buf, int64_t n, void* stream);

/* Gradient buckets over one flat fp32 gradient buffer laid out by parameter-table row:
 * row_offset[i] / row_numel[i] (elements) for the n_rows rows of cfm_encoder_param_name order
 * (numel 0 = no gradient), then any further gradients up to flat_numel (e.g. a CTC head).
 * Pass cfm_grad_buckets_ready_cb / the bucket handle as cfm_train_opts.grad_ready / grad_ready_user:
 * each reported range is all-reduced immediately (ordered after the backward's stream); then
 * cfm_grad_buckets_finish reduces everything not reported yet and scales the whole buffer.
 * One backward per finish writes the buffer from zero.  Gradient accumulation (a second backward of
 * the same step adding into the reduced buffer) is exact with average = 1; with average = 0 scale the
 * buffer by 1/world (cfm_allreduce_grads-free: any device scale) before the second backward, or the
 * already-reduced part comes back world times (conformer_amd/dist.py GradBuckets.attach does this). */
cfm_status cfm_grad_buckets_create(cfm_comm* comm, float* flat, int64_t flat_numel, int n_rows,
                                   const int64_t* row_offset, const int64_t* row_numel, int average,
                                   cfm_grad_buckets** out);
int cfm_grad_buckets_ready_cb(void* user, int first_param, int n_params, void* stream);
cfm_status cfm_grad_buckets_finish(cfm_grad_buckets* b, void* stream);
/* number of all-reduces issued since the last finish (reported ranges + the finish's remainder) */
int cfm_grad_buckets_issued(const cfm_grad_buckets* b);
cfm_status cfm_grad_buckets_destroy(cfm_grad_buckets* b);

#ifdef __cplusplus
}
#endif
#endif
