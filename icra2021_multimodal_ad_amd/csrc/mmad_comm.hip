// Native RCCL gradient exchange for the data-parallel train step
// (replaces the reference's single-process optimizer step,
// novelty_detection.py:90, with a sum all-reduce of per-layer gradient
// buckets over xGMI, overlapped with the rest of the backward).
//
// RCCL is resolved at run time from the copy already loaded in the process
// (torch's librccl.so.1, same soname as /opt/rocm/lib's), falling back to
// dlopen: one RCCL instance per process, no link-time dependency.
#include <dlfcn.h>
#include <cstring>
#include <mutex>

#include <rccl/rccl.h>

#include "mmad_common.h"
#include "mmad_comm.h"

namespace {
struct RcclApi {
  ncclResult_t (*get_unique_id)(ncclUniqueId*);
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int);
  ncclResult_t (*comm_destroy)(ncclComm_t);
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t);
  ncclResult_t (*reduce_scatter)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                                 hipStream_t);
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
  ncclResult_t (*group_start)();
  ncclResult_t (*group_end)();
  const char* (*error_string)(ncclResult_t);
  bool ok;
};

const RcclApi& rccl() {
  static RcclApi api{};
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = RTLD_DEFAULT;
    if (!dlsym(h, "ncclAllReduce")) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
    api.get_unique_id = (decltype(api.get_unique_id))dlsym(h, "ncclGetUniqueId");
    api.comm_init_rank = (decltype(api.comm_init_rank))dlsym(h, "ncclCommInitRank");
    api.comm_destroy = (decltype(api.comm_destroy))dlsym(h, "ncclCommDestroy");
    api.all_reduce = (decltype(api.all_reduce))dlsym(h, "ncclAllReduce");
    api.reduce_scatter = (decltype(api.reduce_scatter))dlsym(h, "ncclReduceScatter");
    api.all_gather = (decltype(api.all_gather))dlsym(h, "ncclAllGather");
    api.error_string = (decltype(api.error_string))dlsym(h, "ncclGetErrorString");
    api.group_start = (decltype(api.group_start))dlsym(h, "ncclGroupStart");
    api.group_end = (decltype(api.group_end))dlsym(h, "ncclGroupEnd");
    api.ok = api.get_unique_id && api.comm_init_rank && api.comm_destroy && api.all_reduce &&
             api.reduce_scatter && api.all_gather && api.error_string && api.group_start &&
             api.group_end;
  });
  return api;
}
}  // namespace

struct mmad_comm {
  ncclComm_t comm = nullptr;
  int rank = 0, nranks = 1;
  float loopback = 0.f;   // > 0: single-GPU loopback, all-reduce = scale by this
};

namespace {
// loopback "all-reduce": buf *= s, after a short delay so that a missing
// dependency on the producer of buf shows up as a wrong result.  A small grid
// (<= 256 workgroups, one per CU) whose waves sleep through the delay (s_sleep, no issue
// pressure) and then scale: one launch, like an RCCL call, and it does not
// hold the chip the way a spin in every block of a full grid did (that stood
// in for an exchange far heavier than RCCL's few channel workgroups)
__global__ void loopback_k(float* __restrict__ buf, int64_t n, float s) {
  const long long t0 = clock64();
  while (clock64() - t0 < 20000) __builtin_amdgcn_s_sleep(8);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    buf[i] *= s;
}
// the same on bf16 (RCCL's bf16 sum rounds each result to bf16: so does this)
__global__ void loopback_bf16_k(bf16* __restrict__ buf, int64_t n, float s) {
  const long long t0 = clock64();
  while (clock64() - t0 < 20000) __builtin_amdgcn_s_sleep(8);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    buf[i] = (bf16)((float)buf[i] * s);
}
}  // namespace

#define MMAD_RCCL_CHECK(expr)                                                        \
  do {                                                                               \
    ncclResult_t r_ = (expr);                                                        \
    if (r_ != ncclSuccess) {                                                         \
      mmad_set_error("RCCL error %s at %s:%d", rccl().error_string(r_), __FILE__, __LINE__); \
      return MMAD_ERCCL;                                                             \
    }                                                                                \
  } while (0)

int mmad_comm_unique_id_bytes(void) { return (int)sizeof(ncclUniqueId); }

int mmad_comm_get_unique_id(void* out) {
  MMAD_CHECK_ARG(out, "comm_get_unique_id: null output");
  MMAD_CHECK_ARG(rccl().ok, "RCCL not available in this process");
  ncclUniqueId id;
  MMAD_RCCL_CHECK(rccl().get_unique_id(&id));
  memcpy(out, &id, sizeof(id));
  return MMAD_OK;
}

int mmad_comm_create(mmad_comm** out, const void* unique_id, int nranks, int rank) {
  MMAD_CHECK_ARG(out && unique_id, "comm_create: null argument");
  MMAD_CHECK_ARG(nranks >= 1 && rank >= 0 && rank < nranks, "comm_create: bad rank %d of %d", rank,
                 nranks);
  MMAD_CHECK_ARG(rccl().ok, "RCCL not available in this process");
  ncclUniqueId id;
  memcpy(&id, unique_id, sizeof(id));
  mmad_comm* c = new mmad_comm;
  c->rank = rank;
  c->nranks = nranks;
  const ncclResult_t r = rccl().comm_init_rank(&c->comm, nranks, id, rank);
  if (r != ncclSuccess) {
    mmad_set_error("RCCL ncclCommInitRank: %s", rccl().error_string(r));
    delete c;
    return MMAD_ERCCL;
  }
  *out = c;
  return MMAD_OK;
}

int mmad_comm_create_loopback(mmad_comm** out, float scale) {
  return mmad_comm_create_loopback_ranks(out, scale, 1, 0);
}

int mmad_comm_create_loopback_ranks(mmad_comm** out, float scale, int nranks, int rank) {
  MMAD_CHECK_ARG(out && scale > 0.f && nranks >= 1 && rank >= 0 && rank < nranks,
                 "comm_create_loopback: bad arguments");
  mmad_comm* c = new mmad_comm;
  c->loopback = scale;
  c->nranks = nranks;
  c->rank = rank;
  *out = c;
  return MMAD_OK;
}

void mmad_comm_destroy(mmad_comm* c) {
  if (!c) return;
  if (c->comm && rccl().ok) (void)rccl().comm_destroy(c->comm);
  delete c;
}

int mmad_allreduce_bucket(mmad_comm* c, float* buf, int64_t n, void* stream) {
  MMAD_CHECK_ARG(c && (buf || n == 0) && n >= 0, "allreduce_bucket: bad arguments");
  if (n == 0) return MMAD_OK;
  if (c->loopback > 0.f) {
    const int64_t blocks = (n + 255) / 256 < 256 ? (n + 255) / 256 : 256;
    loopback_k<<<(int)blocks, 256, 0, (hipStream_t)stream>>>(buf, n, c->loopback);
    MMAD_LAUNCH_CHECK();
    return MMAD_OK;
  }
  MMAD_RCCL_CHECK(rccl().all_reduce(buf, buf, (size_t)n, ncclFloat32, ncclSum, c->comm,
                                    (hipStream_t)stream));
  return MMAD_OK;
}

int mmad_allreduce_pair(mmad_comm* c, float* a, int64_t na, float* b, int64_t nb, void* stream) {
  MMAD_CHECK_ARG(c && (a || na == 0) && (b || nb == 0) && na >= 0 && nb >= 0, "allreduce_pair: bad arguments");
  if (c->loopback > 0.f) {
    const int rc = mmad_allreduce_bucket(c, a, na, stream);
    return rc != MMAD_OK ? rc : mmad_allreduce_bucket(c, b, nb, stream);
  }
  MMAD_RCCL_CHECK(rccl().group_start());
  ncclResult_t r = na ? rccl().all_reduce(a, a, (size_t)na, ncclFloat32, ncclSum, c->comm, (hipStream_t)stream)
                      : ncclSuccess;
  if (r == ncclSuccess && nb)
    r = rccl().all_reduce(b, b, (size_t)nb, ncclFloat32, ncclSum, c->comm, (hipStream_t)stream);
  const ncclResult_t e = rccl().group_end();   // always close the group
  MMAD_RCCL_CHECK(r);
  MMAD_RCCL_CHECK(e);
  return MMAD_OK;
}

int mmad_comm_size(const mmad_comm* c) { return c ? c->nranks : 0; }
int mmad_comm_rank(const mmad_comm* c) { return c ? c->rank : -1; }

// Sharded exchange (the data-parallel step's ZeRO-1 form: each rank updates
// the Adam state of its 1/N of a bucket).  In place, RCCL's own in-place
// convention: rank r's shard is buf[r*n/N, (r+1)*n/N).
int mmad_reduce_scatter_bucket(mmad_comm* c, float* buf, int64_t n, void* stream) {
  MMAD_CHECK_ARG(c && (buf || n == 0) && n >= 0, "reduce_scatter_bucket: bad arguments");
  MMAD_CHECK_ARG(n % c->nranks == 0, "reduce_scatter_bucket: n=%lld not divisible by %d ranks",
                 (long long)n, c->nranks);
  if (n == 0) return MMAD_OK;
  const size_t cnt = (size_t)(n / c->nranks);
  // loopback posing as rank r of N: like RCCL's in-place reduce-scatter, only
  // this rank's slice [r * n / N, (r + 1) * n / N) receives the reduced values
  if (c->loopback > 0.f) return mmad_allreduce_bucket(c, buf + (size_t)c->rank * cnt, (int64_t)cnt, stream);
  MMAD_RCCL_CHECK(rccl().reduce_scatter(buf, buf + (size_t)c->rank * cnt, cnt, ncclFloat32, ncclSum,
                                        c->comm, (hipStream_t)stream));
  return MMAD_OK;
}

// the same on a bf16 buffer (the optional bf16 gradient exchange: half the bytes)
int mmad_reduce_scatter_bucket_bf16(mmad_comm* c, void* buf, int64_t n, void* stream) {
  MMAD_CHECK_ARG(c && (buf || n == 0) && n >= 0, "reduce_scatter_bucket_bf16: bad arguments");
  MMAD_CHECK_ARG(n % c->nranks == 0, "reduce_scatter_bucket_bf16: n=%lld not divisible by %d ranks",
                 (long long)n, c->nranks);
  if (n == 0) return MMAD_OK;
  const size_t cnt = (size_t)(n / c->nranks);
  bf16* b = (bf16*)buf;
  if (c->loopback > 0.f) {
    const int64_t blocks = ((int64_t)cnt + 255) / 256 < 256 ? ((int64_t)cnt + 255) / 256 : 256;
    loopback_bf16_k<<<(int)blocks, 256, 0, (hipStream_t)stream>>>(b + (size_t)c->rank * cnt, (int64_t)cnt,
                                                                   c->loopback);
    MMAD_LAUNCH_CHECK();
    return MMAD_OK;
  }
  MMAD_RCCL_CHECK(rccl().reduce_scatter(b, b + (size_t)c->rank * cnt, cnt, ncclBfloat16, ncclSum, c->comm,
                                        (hipStream_t)stream));
  return MMAD_OK;
}

int mmad_all_gather_bucket(mmad_comm* c, void* buf, int64_t n, int dtype, void* stream) {
  MMAD_CHECK_ARG(c && (buf || n == 0) && n >= 0, "all_gather_bucket: bad arguments");
  MMAD_CHECK_ARG(dtype == MMAD_F32 || dtype == MMAD_BF16, "all_gather_bucket: bad dtype %d", dtype);
  MMAD_CHECK_ARG(n % c->nranks == 0, "all_gather_bucket: n=%lld not divisible by %d ranks", (long long)n,
                 c->nranks);
  if (n == 0 || c->loopback > 0.f || c->nranks == 1) return MMAD_OK;   // one rank holds every shard
  const size_t cnt = (size_t)(n / c->nranks);
  const size_t es = dtype == MMAD_BF16 ? 2 : 4;
  MMAD_RCCL_CHECK(rccl().all_gather((const char*)buf + (size_t)c->rank * cnt * es, buf, cnt,
                                    dtype == MMAD_BF16 ? ncclBfloat16 : ncclFloat32, c->comm,
                                    (hipStream_t)stream));
  return MMAD_OK;
}
