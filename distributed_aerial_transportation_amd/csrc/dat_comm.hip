// dat_comm.hip -- the metric collectives of a sharded run over RCCL (kernel K8 of SURVEY.md 8(e)), part of
// libdat.so's C-ABI (include/dat.h: dat_comm_*).
//
// Closed-loop scenarios are independent, so nothing crosses GPUs inside a control step; a sharded run (one
// process per GPU) exchanges only the per-scenario metrics the reference keeps in its loop's lists (iteration
// counts, min env distance, collision flag: example/rqp_example.py:112-138) and the run's work counters.
// Those go over RCCL (xGMI between the GPUs of a node) directly from the C-ABI: no PyTorch in the rank
// processes.  Host buffers in and out; each call stages them through device buffers of the communicator's
// device and synchronises its stream.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>

#include "../../include/dat.h"

struct dat_comm {
  int device = 0, nranks = 1, rank = 0;
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;
  double* dbuf = nullptr;  // send area [cap], then recv area [nranks cap]
  size_t cap = 0;
};

namespace {

thread_local std::string g_comm_err;

int cfail(const std::string& m) {
  g_comm_err = m;
  return -1;
}

#define HIPC(x)                                                                            \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) return cfail(std::string(#x) + ": " + hipGetErrorString(e_));    \
  } while (0)
#define NCCLC(x)                                                                           \
  do {                                                                                     \
    ncclResult_t r_ = (x);                                                                 \
    if (r_ != ncclSuccess) return cfail(std::string(#x) + ": " + ncclGetErrorString(r_)); \
  } while (0)

// device staging buffer for `count` doubles sent by each rank
int reserve(dat_comm* c, size_t count) {
  if (count <= c->cap) return 0;
  if (c->dbuf) HIPC(hipFree(c->dbuf));
  c->dbuf = nullptr;
  c->cap = 0;
  HIPC(hipMalloc((void**)&c->dbuf, sizeof(double) * count * (size_t)(c->nranks + 1)));
  c->cap = count;
  return 0;
}

}  // namespace

extern "C" {

const char* dat_comm_last_error(void) { return g_comm_err.c_str(); }

int dat_comm_unique_id(unsigned char* id) {
  if (!id) return cfail("dat_comm_unique_id: null argument");
  ncclUniqueId u;
  NCCLC(ncclGetUniqueId(&u));
  static_assert(sizeof(u) == DAT_COMM_ID_BYTES, "RCCL unique id size");
  memcpy(id, &u, sizeof(u));
  return 0;
}

int dat_comm_create(int device, int nranks, int rank, const unsigned char* id, dat_comm** out) {
  if (!id || !out) return cfail("dat_comm_create: null argument");
  *out = nullptr;
  if (nranks < 1 || rank < 0 || rank >= nranks) return cfail("dat_comm_create: rank out of range");
  HIPC(hipSetDevice(device));
  dat_comm* c = new dat_comm();
  c->device = device;
  c->nranks = nranks;
  c->rank = rank;
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return cfail("dat_comm_create: stream creation failed");
  }
  const ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);  // collective over the nranks processes
  if (r != ncclSuccess) {
    (void)hipStreamDestroy(c->stream);
    delete c;
    return cfail(std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  }
  *out = c;
  return 0;
}

int dat_comm_destroy(dat_comm* c) {
  if (!c) return 0;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->comm) (void)ncclCommDestroy(c->comm);
  if (c->dbuf) (void)hipFree(c->dbuf);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  return 0;
}

int dat_comm_allgather(dat_comm* c, const double* send, long long count, double* recv) {
  if (!c || (count > 0 && (!send || !recv))) return cfail("dat_comm_allgather: null argument");
  if (count < 0) return cfail("dat_comm_allgather: negative count");
  if (count == 0) return 0;
  HIPC(hipSetDevice(c->device));
  if (reserve(c, (size_t)count)) return -1;
  double* ds = c->dbuf;
  double* dr = c->dbuf + c->cap;
  HIPC(hipMemcpyAsync(ds, send, sizeof(double) * count, hipMemcpyHostToDevice, c->stream));
  NCCLC(ncclAllGather(ds, dr, (size_t)count, ncclDouble, c->comm, c->stream));
  HIPC(hipMemcpyAsync(recv, dr, sizeof(double) * count * c->nranks, hipMemcpyDeviceToHost, c->stream));
  HIPC(hipStreamSynchronize(c->stream));
  return 0;
}

int dat_comm_allreduce(dat_comm* c, double* buf, long long count, int op) {
  if (!c || (count > 0 && !buf)) return cfail("dat_comm_allreduce: null argument");
  if (op != DAT_COMM_SUM && op != DAT_COMM_MAX) return cfail("dat_comm_allreduce: op is DAT_COMM_SUM or DAT_COMM_MAX");
  if (count < 0) return cfail("dat_comm_allreduce: negative count");
  if (count == 0) return 0;
  HIPC(hipSetDevice(c->device));
  if (reserve(c, (size_t)count)) return -1;
  HIPC(hipMemcpyAsync(c->dbuf, buf, sizeof(double) * count, hipMemcpyHostToDevice, c->stream));
  NCCLC(ncclAllReduce(c->dbuf, c->dbuf, (size_t)count, ncclDouble, op == DAT_COMM_SUM ? ncclSum : ncclMax, c->comm,
                      c->stream));
  HIPC(hipMemcpyAsync(buf, c->dbuf, sizeof(double) * count, hipMemcpyDeviceToHost, c->stream));
  HIPC(hipStreamSynchronize(c->stream));
  return 0;
}

int dat_comm_barrier(dat_comm* c) {
  if (!c) return cfail("dat_comm_barrier: null communicator");
  HIPC(hipSetDevice(c->device));
  HIPC(hipDeviceSynchronize());  // every stream of this process (the handles' kernels) has drained
  double one = 1.0;
  return dat_comm_allreduce(c, &one, 1, DAT_COMM_SUM);
}

}  // extern "C"
