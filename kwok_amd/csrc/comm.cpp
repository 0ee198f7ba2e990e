// The reporting interval's cluster-aggregate all-reduce over RCCL (xGMI), for a non-Python host:
// include/kwok_comm.h.  Host code only (no kernels): RCCL does the transfer on its own stream,
// ordered against the engines' streams with HIP events.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>
#include <vector>

#include "../../include/kwok_comm.h"
#include "../../include/kwok_engine.h"

struct kwk_comm {
  int device = 0;
  int rank = 0, world = 1;
  ncclComm_t nccl = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;              // the last all-reduce on `stream`
  std::vector<hipEvent_t> joins;          // one per engine stream joined
  double* buf = nullptr;
  uint64_t cap = 0;
  std::string err;
};

namespace {

thread_local std::string g_err;
thread_local std::string* tl_err = nullptr;
struct ErrScope {
  std::string* prev;
  explicit ErrScope(kwk_comm* c) : prev(tl_err) { tl_err = c ? &c->err : nullptr; }
  ~ErrScope() { tl_err = prev; }
};
kwk_status fail(kwk_status code, const std::string& msg) {
  g_err = msg;
  if (tl_err) *tl_err = msg;
  return code;
}

#define HIP_OK(x)                                                                                   \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) return fail(KWK_EHIP, std::string(#x) + ": " + hipGetErrorString(e_));    \
  } while (0)
#define NCCL_OK(x)                                                                                  \
  do {                                                                                              \
    ncclResult_t r_ = (x);                                                                          \
    if (r_ != ncclSuccess) return fail(KWK_EHIP, std::string(#x) + ": " + ncclGetErrorString(r_));  \
  } while (0)

}  // namespace

extern "C" {

const char* kwk_comm_last_error(const kwk_comm* c) { return c ? c->err.c_str() : g_err.c_str(); }

kwk_status kwk_comm_unique_id(uint8_t id[KWK_COMM_ID_BYTES]) {
  if (!id) return fail(KWK_EINVAL, "null argument");
  ncclUniqueId u;
  NCCL_OK(ncclGetUniqueId(&u));
  static_assert(sizeof(u) == KWK_COMM_ID_BYTES, "ncclUniqueId size");
  memcpy(id, &u, sizeof(u));
  return KWK_OK;
}

kwk_status kwk_comm_init(const uint8_t id[KWK_COMM_ID_BYTES], int32_t rank, int32_t world, int32_t device,
                         kwk_comm** out) {
  if (!id || !out) return fail(KWK_EINVAL, "null argument");
  if (world < 1 || rank < 0 || rank >= world) return fail(KWK_EINVAL, "rank / world out of range");
  int ndev = 0;
  HIP_OK(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(KWK_EINVAL, "device ordinal out of range");
  HIP_OK(hipSetDevice(device));
  auto* c = new kwk_comm();
  c->device = device;
  c->rank = rank;
  c->world = world;
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclResult_t r = ncclCommInitRank(&c->nccl, world, u, rank);
  if (r != ncclSuccess) {
    delete c;
    return fail(KWK_EHIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  }
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->done, hipEventDisableTiming) != hipSuccess) {
    kwk_comm_destroy(c);
    return fail(KWK_EHIP, "stream / event creation");
  }
  *out = c;
  return KWK_OK;
}

kwk_status kwk_comm_destroy(kwk_comm* c) {
  if (!c) return KWK_OK;
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  if (c->nccl) ncclCommDestroy(c->nccl);
  if (c->buf) hipFree(c->buf);
  for (hipEvent_t e : c->joins) hipEventDestroy(e);
  if (c->done) hipEventDestroy(c->done);
  if (c->stream) hipStreamDestroy(c->stream);
  delete c;
  return KWK_OK;
}

kwk_status kwk_comm_buffer(kwk_comm* c, uint64_t n, double** dev) {
  ErrScope es_(c);
  if (!c || !dev) return fail(KWK_EINVAL, "null argument");
  HIP_OK(hipSetDevice(c->device));
  if (n > c->cap) {
    HIP_OK(hipStreamSynchronize(c->stream));
    if (c->buf) HIP_OK(hipFree(c->buf));
    c->buf = nullptr;
    HIP_OK(hipMalloc(&c->buf, 8 * n));
    // zeroed on the communicator's stream and complete on return: the engines write into the
    // buffer from their own non-blocking streams, which would not wait for a null-stream memset
    HIP_OK(hipMemsetAsync(c->buf, 0, 8 * n, c->stream));
    HIP_OK(hipStreamSynchronize(c->stream));
    c->cap = n;
  }
  *dev = c->buf;
  return KWK_OK;
}

kwk_status kwk_comm_allreduce(kwk_comm* c, uint64_t n, kwk_engine* const* engines, uint32_t n_engines) {
  ErrScope es_(c);
  if (!c || (n_engines && !engines)) return fail(KWK_EINVAL, "null argument");
  if (n > c->cap) return fail(KWK_EINVAL, "n beyond the communicator's buffer (kwk_comm_buffer)");
  HIP_OK(hipSetDevice(c->device));
  while (c->joins.size() < n_engines) {
    hipEvent_t e;
    HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c->joins.push_back(e);
  }
  std::vector<hipStream_t> streams(n_engines);
  for (uint32_t i = 0; i < n_engines; ++i) {  // the collective waits for every engine's queued work
    void* s = nullptr;
    if (kwk_stream(engines[i], &s) != KWK_OK) return fail(KWK_EINVAL, "engine " + std::to_string(i) + ": kwk_stream");
    streams[i] = (hipStream_t)s;
    HIP_OK(hipEventRecord(c->joins[i], streams[i]));
    HIP_OK(hipStreamWaitEvent(c->stream, c->joins[i], 0));
  }
  if (n) NCCL_OK(ncclAllReduce(c->buf, c->buf, (size_t)n, ncclFloat64, ncclSum, c->nccl, c->stream));
  HIP_OK(hipEventRecord(c->done, c->stream));
  for (uint32_t i = 0; i < n_engines; ++i) HIP_OK(hipStreamWaitEvent(streams[i], c->done, 0));
  return KWK_OK;
}

kwk_status kwk_comm_read(kwk_comm* c, double* host_out, uint64_t n) {
  ErrScope es_(c);
  if (!c || (n && !host_out)) return fail(KWK_EINVAL, "null argument");
  if (n > c->cap) return fail(KWK_EINVAL, "n beyond the communicator's buffer");
  HIP_OK(hipSetDevice(c->device));
  if (n) HIP_OK(hipMemcpyAsync(host_out, c->buf, 8 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_OK(hipStreamSynchronize(c->stream));
  return KWK_OK;
}

}  // extern "C"
