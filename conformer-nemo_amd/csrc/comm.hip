// Data-parallel communication through the C-ABI (include/cfm_comm.h).
//
// RCCL entry points are resolved with dlsym when the first communicator is created: first from
// the process (a PyTorch-ROCm process has its RCCL loaded already), else from librccl.so.1, so
// libcfm.so has no link-time RCCL dependency and never loads a second RCCL next to torch's.
//
// Overlap: a gradient bucket owns a communication stream.  grad_ready (called by
// cfm_train_backward while it enqueues) records an event on the backward's stream, makes the comm
// stream wait on it and enqueues the bucket's ncclAllReduce there, so the reduction of layer l runs
// while layers l-1 .. 0 compute.  finish() reduces the rest, makes the caller's stream wait for the
// comm stream and scales the whole buffer once (DDP averaging).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "../../include/cfm_comm.h"
#include "cfm_abi.h"
#include "cfm_kernels.h"

namespace cfm {
namespace {

struct Rccl {
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

const Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  static std::string err;
  std::call_once(once, [] {
    void* h = RTLD_DEFAULT;
    if (!dlsym(h, "ncclAllReduce")) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      err = "RCCL not found (librccl.so.1)";
      return;
    }
    r.get_unique_id = (decltype(r.get_unique_id))dlsym(h, "ncclGetUniqueId");
    r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(h, "ncclCommInitRank");
    r.all_reduce = (decltype(r.all_reduce))dlsym(h, "ncclAllReduce");
    r.comm_destroy = (decltype(r.comm_destroy))dlsym(h, "ncclCommDestroy");
    r.error_string = (decltype(r.error_string))dlsym(h, "ncclGetErrorString");
  });
  if (!r.all_reduce || !r.comm_init_rank || !r.get_unique_id || !r.comm_destroy)
    fail(CFM_ERR_UNSUPPORTED, err.empty() ? "RCCL symbols not found" : err);
  return r;
}

void nccl_ok(ncclResult_t res, const char* what) {
  if (res != ncclSuccess) {
    const Rccl& r = rccl();
    fail(CFM_ERR_HIP, std::string(what) + ": " + (r.error_string ? r.error_string(res) : "RCCL error"));
  }
}

__global__ void scale_kernel(float* __restrict__ x, long n, float s) {
  const long n4 = n / 4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    float4 v = ((float4*)x)[i];
    v.x *= s; v.y *= s; v.z *= s; v.w *= s;
    ((float4*)x)[i] = v;
  }
  for (long i = 4 * n4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) x[i] *= s;
}

void scale(float* x, long n, float s, hipStream_t st) {
  if (n <= 0 || s == 1.0f) return;
  if (((uintptr_t)x & 15) != 0) fail(CFM_ERR_INVALID_ARG, "gradient buffer must be 16-byte aligned");
  const long blocks = std::min<long>((n / 4 + 255) / 256 + 1, 4096);
  cfm_launch(scale_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, n, s);
}

}  // namespace
}  // namespace cfm

struct cfm_comm {
  ncclComm_t nc = nullptr;
  int rank = 0, world = 1, device = 0;
};

struct cfm_grad_buckets {
  cfm_comm* comm = nullptr;
  float* flat = nullptr;
  int64_t numel = 0;
  std::vector<int64_t> off, cnt;   // per table row
  bool average = true;
  hipStream_t cs = nullptr;        // communication stream
  hipEvent_t ev_ready = nullptr, ev_done = nullptr;
  std::vector<std::pair<int64_t, int64_t>> issued;   // [start, end) since the last finish
};

using namespace cfm;

namespace {
void bucket_issue(cfm_grad_buckets* b, int64_t start, int64_t end, hipStream_t producer) {
  if (end <= start) return;
  b->issued.push_back({start, end});
  HIP_OK(hipEventRecord(b->ev_ready, producer));
  HIP_OK(hipStreamWaitEvent(b->cs, b->ev_ready, 0));
  float* p = b->flat + start;
  nccl_ok(rccl().all_reduce(p, p, (size_t)(end - start), ncclFloat32, ncclSum, b->comm->nc, b->cs), "ncclAllReduce");
}
}  // namespace

extern "C" {

cfm_status cfm_comm_get_unique_id(char unique_id[CFM_COMM_ID_BYTES]) {
  return guarded([&] {
    if (!unique_id) fail(CFM_ERR_INVALID_ARG, "null argument");
    ncclUniqueId id;
    nccl_ok(rccl().get_unique_id(&id), "ncclGetUniqueId");
    static_assert(sizeof(id) == CFM_COMM_ID_BYTES, "unique id size");
    std::memcpy(unique_id, &id, sizeof(id));
  });
}

cfm_status cfm_comm_init(int rank, int world, const char unique_id[CFM_COMM_ID_BYTES], int device, cfm_comm** out) {
  return guarded([&] {
    if (!unique_id || !out || world < 1 || rank < 0 || rank >= world) fail(CFM_ERR_INVALID_ARG, "bad communicator arguments");
    *out = nullptr;
    int prev = 0;
    HIP_OK(hipGetDevice(&prev));
    HIP_OK(hipSetDevice(device));
    ncclUniqueId id;
    std::memcpy(&id, unique_id, sizeof(id));
    auto c = new cfm_comm;
    c->rank = rank;
    c->world = world;
    c->device = device;
    const ncclResult_t r = rccl().comm_init_rank(&c->nc, world, id, rank);
    (void)hipSetDevice(prev);
    if (r != ncclSuccess) {
      delete c;
      nccl_ok(r, "ncclCommInitRank");
    }
    *out = c;
  });
}

cfm_status cfm_comm_destroy(cfm_comm* comm) {
  return guarded([&] {
    if (!comm) return;
    if (comm->nc) nccl_ok(rccl().comm_destroy(comm->nc), "ncclCommDestroy");
    delete comm;
  });
}

int cfm_comm_world(const cfm_comm* comm) { return comm ? comm->world : 0; }

cfm_status cfm_allreduce_grads(cfm_comm* comm, float* buf, int64_t n, float scale_by, void* stream) {
  return guarded([&] {
    if (!comm || (!buf && n > 0) || n < 0) fail(CFM_ERR_INVALID_ARG, "bad all-reduce arguments");
    if (n == 0) return;
    hipStream_t st = (hipStream_t)stream;
    nccl_ok(rccl().all_reduce(buf, buf, (size_t)n, ncclFloat32, ncclSum, comm->nc, st), "ncclAllReduce");
    scale(buf, n, scale_by, st);
  });
}

int cfm_comm_allreduce_cb(void* user, float* buf, int64_t n, void* stream) {
  return cfm_allreduce_grads((cfm_comm*)user, buf, n, 1.0f, stream) == CFM_OK ? 0 : 1;
}

cfm_status cfm_grad_buckets_create(cfm_comm* comm, float* flat, int64_t flat_numel, int n_rows,
                                   const int64_t* row_offset, const int64_t* row_numel, int average,
                                   cfm_grad_buckets** out) {
  return guarded([&] {
    if (!comm || !flat || flat_numel <= 0 || n_rows < 0 || (n_rows && (!row_offset || !row_numel)) || !out)
      fail(CFM_ERR_INVALID_ARG, "bad bucket arguments");
    *out = nullptr;
    auto b = new cfm_grad_buckets;
    b->comm = comm;
    b->flat = flat;
    b->numel = flat_numel;
    b->average = average != 0;
    b->off.assign(row_offset, row_offset + n_rows);
    b->cnt.assign(row_numel, row_numel + n_rows);
    for (int i = 0; i < n_rows; ++i)
      if (b->cnt[i] < 0 || (b->cnt[i] > 0 && (b->off[i] < 0 || b->off[i] + b->cnt[i] > flat_numel))) {
        delete b;
        fail(CFM_ERR_INVALID_ARG, "bucket row outside the gradient buffer");
      }
    {   // rows must not overlap: an element in two rows would be all-reduced twice
      std::vector<std::pair<int64_t, int64_t>> r;
      for (int i = 0; i < n_rows; ++i)
        if (b->cnt[i] > 0) r.push_back({b->off[i], b->off[i] + b->cnt[i]});
      std::sort(r.begin(), r.end());
      for (size_t i = 1; i < r.size(); ++i)
        if (r[i].first < r[i - 1].second) {
          delete b;
          fail(CFM_ERR_INVALID_ARG, "bucket rows overlap in the gradient buffer");
        }
    }
    int prev = 0;
    HIP_OK(hipGetDevice(&prev));
    HIP_OK(hipSetDevice(comm->device));
    HIP_OK(hipStreamCreateWithFlags(&b->cs, hipStreamNonBlocking));
    HIP_OK(hipEventCreateWithFlags(&b->ev_ready, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&b->ev_done, hipEventDisableTiming));
    (void)hipSetDevice(prev);
    *out = b;
  });
}

int cfm_grad_buckets_ready_cb(void* user, int first_param, int n_params, void* stream) {
  auto* b = (cfm_grad_buckets*)user;
  const cfm_status s = guarded([&] {
    if (!b) fail(CFM_ERR_INVALID_ARG, "null bucket handle");
    // the reported rows' byte ranges, merged into maximal contiguous runs: one all-reduce per run, so
    // a layout whose rows are not adjacent never pulls in (and double-reduces) another row's slice
    std::vector<std::pair<int64_t, int64_t>> spans;
    for (int i = std::max(first_param, 0); i < first_param + n_params && i < (int)b->off.size(); ++i)
      if (b->cnt[i] > 0) spans.push_back({b->off[i], b->off[i] + b->cnt[i]});
    std::sort(spans.begin(), spans.end());
    for (size_t i = 0; i < spans.size();) {
      int64_t lo = spans[i].first, hi = spans[i].second;
      size_t j = i + 1;
      while (j < spans.size() && spans[j].first == hi) hi = spans[j++].second;
      bucket_issue(b, lo, hi, (hipStream_t)stream);
      i = j;
    }
  });
  return s == CFM_OK ? 0 : 1;
}

cfm_status cfm_grad_buckets_finish(cfm_grad_buckets* b, void* stream) {
  return guarded([&] {
    if (!b) fail(CFM_ERR_INVALID_ARG, "null bucket handle");
    hipStream_t st = (hipStream_t)stream;
    std::vector<std::pair<int64_t, int64_t>> cov = b->issued;
    std::sort(cov.begin(), cov.end());
    int64_t pos = 0;
    std::vector<std::pair<int64_t, int64_t>> gaps;
    for (auto& r : cov) {
      if (r.first > pos) gaps.push_back({pos, r.first});
      pos = std::max(pos, r.second);
    }
    if (pos < b->numel) gaps.push_back({pos, b->numel});
    for (auto& g : gaps) bucket_issue(b, g.first, g.second, st);
    HIP_OK(hipEventRecord(b->ev_done, b->cs));
    HIP_OK(hipStreamWaitEvent(st, b->ev_done, 0));
    if (b->average) scale(b->flat, b->numel, 1.0f / (float)b->comm->world, st);
    b->issued.clear();
  });
}

int cfm_grad_buckets_issued(const cfm_grad_buckets* b) { return b ? (int)b->issued.size() : -1; }

cfm_status cfm_grad_buckets_destroy(cfm_grad_buckets* b) {
  return guarded([&] {
    if (!b) return;
    if (b->cs) (void)hipStreamDestroy(b->cs);
    if (b->ev_ready) (void)hipEventDestroy(b->ev_ready);
    if (b->ev_done) (void)hipEventDestroy(b->ev_done);
    delete b;
  });
}

}  // extern "C"
